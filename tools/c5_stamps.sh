# per-phase stamps of the deep-tier kernels at the C5 shape (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python tools/stamps_glob.py 4 1000000 2000 dense > gpurun_out/stamps_glob_c5.txt 2>&1 && \
timeout -k 10 300 python tools/stamps_diff.py 8 1000000 2000 > gpurun_out/stamps_diff_c5.txt 2>&1
echo rc=$?
