# temporary experiment driver (GPU box)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/prof_bench.sh r03z_c5 --config c5 --steps 3 --warmup 1
