# per-phase stamps of k_build and k_chains at the C3 shape (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python tools/stamps_build.py 5000 > gpurun_out/stamps_build_c3.txt 2>&1 && \
timeout -k 10 300 python tools/stamps_chains.py 5000 > gpurun_out/stamps_chains_c3.txt 2>&1
