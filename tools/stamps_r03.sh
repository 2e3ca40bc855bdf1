# per-phase stamps of k_chains_glob at the C5 shape, both workgroup sizes (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
NEMO_GLOB_BLOCK=256 timeout -k 10 300 python tools/stamps_glob.py 4 1000000 2000 dense > gpurun_out/stamps_glob256.txt 2>&1 && \
NEMO_GLOB_BLOCK=512 timeout -k 10 300 python tools/stamps_glob.py 4 1000000 2000 dense > gpurun_out/stamps_glob512.txt 2>&1
