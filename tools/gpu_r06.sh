#!/bin/bash
# round-6 GPU steps (run under gpurun, one part per call); every GPU step has its own time limit
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${2:-r06}
case "$1" in
new)  # the round's new tests first, then the whole suite
  timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batched.py \
    tests/test_gpu_diff.py tests/test_gpu_parity.py::test_stage_and_diff_streams > gpurun_out/${tag}_new.log 2>&1
  rc=$?; tail -5 gpurun_out/${tag}_new.log; [ $rc -eq 0 ] || exit $rc ;;
suite)
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_suite.log 2>&1
  rc=$?; tail -3 gpurun_out/${tag}_suite.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || exit 1
  tail -1 gpurun_out/${tag}_smoke.log ;;
bench)
  timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${tag}_bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['frac'])" ;;
esac
echo part $1 done
case "$1" in
perrun)
  timeout -k 10 400 python -u bench.py --diff-mode per_run --no-cpu-baseline --e2e-runs 0 > gpurun_out/${tag}_perrun.json 2> gpurun_out/${tag}_perrun.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${tag}_perrun.json'));r=d['roofline_diff'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'])" ;;
c5)
  timeout -k 10 600 python -u bench.py --config c5 --steps 2 --warmup 1 --e2e-runs 0 --no-cpu-baseline > gpurun_out/${tag}_c5.json 2> gpurun_out/${tag}_c5.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${tag}_c5.json'));print(d['value'],d['ms_per_step'],d['roofline_diff']['avg_launch_ms']);[print(k,v) for k,v in d['kernels'].items()]" ;;
esac
case "$1" in
host)
  timeout -k 10 300 python -u tools/step_host.py > gpurun_out/${tag}_host.txt 2>&1 || exit 1
  cat gpurun_out/${tag}_host.txt ;;
trace)
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --e2e-runs 0 --steps 4 --diff-reps 0 > gpurun_out/${tag}_trace.log 2>&1 || exit 1
  python tools/timeline.py $(find gpurun_out/${tag}_trace -name "kt_kernel_trace.csv" | head -1) > gpurun_out/${tag}_timeline.txt || exit 1
  tail -3 gpurun_out/${tag}_timeline.txt ;;
esac
case "$1" in
hostab)
  timeout -k 10 300 python -u tools/step_host.py > gpurun_out/${tag}_hostA.txt 2>&1 || exit 1
  STAGE_FIRST=1 timeout -k 10 300 python -u tools/step_host.py > gpurun_out/${tag}_hostB.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/step_host.py > gpurun_out/${tag}_hostA2.txt 2>&1 || exit 1
  STAGE_FIRST=1 timeout -k 10 300 python -u tools/step_host.py > gpurun_out/${tag}_hostB2.txt 2>&1 || exit 1
  grep "ms per step" gpurun_out/${tag}_host*.txt ;;
esac
case "$1" in
hostab2)
  timeout -k 10 300 python -u tools/step_host.py > gpurun_out/${tag}_hostA.txt 2>&1 || exit 1
  STAGE_FIRST=1 timeout -k 10 300 python -u tools/step_host.py > gpurun_out/${tag}_hostB.txt 2>&1 || exit 1
  NEMO_STAGE_SDMA=1 timeout -k 10 300 python -u tools/step_host.py > gpurun_out/${tag}_hostC.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/step_host.py > gpurun_out/${tag}_hostA2.txt 2>&1 || exit 1
  grep "ms per step" gpurun_out/${tag}_host*.txt ;;
esac
case "$1" in
c5ab)
  timeout -k 10 600 python -u bench.py --config c5 --steps 2 --warmup 1 --e2e-runs 0 --no-cpu-baseline --diff-reps 2 > gpurun_out/${tag}_c5.json 2> gpurun_out/${tag}_c5.err || exit 1
  timeout -k 10 600 python -u bench.py --config c5 --steps 2 --warmup 1 --e2e-runs 0 --no-cpu-baseline --diff-reps 2 --set topo_ell=0 > gpurun_out/${tag}_c5_old.json 2> gpurun_out/${tag}_c5_old.err || exit 1
  for f in gpurun_out/${tag}_c5.json gpurun_out/${tag}_c5_old.json; do python -c "import json,sys;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],{k:v['ms_total'] for k,v in d['kernels'].items() if k in ('k_topo','k_csrb','k_chains','k_proto')})"; done ;;
esac
case "$1" in
timingab)
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-runs 0 --diff-reps 0 > gpurun_out/${tag}_on.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-runs 0 --diff-reps 0 --kernel-timing off > gpurun_out/${tag}_off.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-runs 0 --diff-reps 0 > gpurun_out/${tag}_on2.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-runs 0 --diff-reps 0 --kernel-timing off > gpurun_out/${tag}_off2.json 2>/dev/null || exit 1
  for f in on off on2 off2; do python -c "import json;d=json.load(open('gpurun_out/${tag}_$f.json'));print('$f',d['value'],d['ms_per_step'])"; done ;;
esac
case "$1" in
timingab2)
  for m in dominant on dominant off; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-runs 0 --diff-reps 0 --kernel-timing $m > gpurun_out/${tag}_$m.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_$m.json'));print('$m',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['avg_launch_ms'])"
  done ;;
esac
case "$1" in
benchprev)
  for b in bench_prev.py bench.py bench_prev.py bench.py; do
    timeout -k 10 300 python -u $b --no-cpu-baseline --e2e-runs 0 --diff-reps 0 > gpurun_out/${tag}_x.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_x.json'));print('$b',d['value'],d['ms_per_step'])"
  done ;;
esac
case "$1" in
benchprev2)
  for b in bench_prev.py bench.py bench_prev.py bench.py; do
    timeout -k 10 300 python -u $b --no-cpu-baseline --e2e-runs 0 --diff-reps 0 --kernel-timing off > gpurun_out/${tag}_x.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_x.json'));print('$b',d['value'],d['ms_per_step'],d.get('step_host_ms_rank0'))"
  done ;;
esac
case "$1" in
benchprev3)
  for b in bench_prev.py bench.py bench_v2.py; do
    timeout -k 10 300 python -u $b --no-cpu-baseline --e2e-runs 0 --diff-reps 0 --kernel-timing off > gpurun_out/${tag}_x.json 2>gpurun_out/${tag}_x.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_x.json'));print('$b',d['value'],d['ms_per_step'],d.get('step_host_ms_rank0'))"; grep STEPS gpurun_out/${tag}_x.err || true
  done ;;
esac
case "$1" in
benchprev4)
  for b in bench_v3.py bench_v2.py bench_v3.py; do
    timeout -k 10 300 python -u $b --no-cpu-baseline --e2e-runs 0 --diff-reps 0 --kernel-timing off > gpurun_out/${tag}_x.json 2>gpurun_out/${tag}_x.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_x.json'));print('$b',d['value'],d['ms_per_step'],d.get('step_host_ms_rank0'))"
  done ;;
esac
case "$1" in
benchgc)
  for b in bench.py bench_prev.py bench.py; do
    timeout -k 10 300 python -u $b --no-cpu-baseline --e2e-runs 0 --diff-reps 0 > gpurun_out/${tag}_x.json 2>gpurun_out/${tag}_x.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_x.json'));print('$b',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['frac'],d.get('step_host_ms_rank0'))"; grep STEPS gpurun_out/${tag}_x.err || true
  done ;;
esac
case "$1" in
bisect)
  for b in bench_prev.py bench_va.py bench_vb.py bench_vc.py bench.py; do
    timeout -k 10 300 python -u $b --no-cpu-baseline --e2e-runs 0 --diff-reps 0 > gpurun_out/${tag}_x.json 2>gpurun_out/${tag}_x.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_x.json'));print('$b',d['value'],d['ms_per_step'])"; grep STEPS gpurun_out/${tag}_x.err || true
  done ;;
esac
case "$1" in
bisect2)
  for b in bench_vb.py bench_p1.py bench_p2.py bench_p3.py bench_prev.py bench_vb.py; do
    timeout -k 10 300 python -u $b --no-cpu-baseline --e2e-runs 0 --diff-reps 0 > gpurun_out/${tag}_x.json 2>gpurun_out/${tag}_x.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_x.json'));print('$b',d['value'],d['ms_per_step'])"; grep STEPS gpurun_out/${tag}_x.err | cut -c1-40 || true
  done ;;
esac
case "$1" in
e2eab)  # the e2e leg of round 4's tree and of this one, alternately, on one box
  for t in r04 now r04 now; do
    if [ $t = r04 ]; then d=var/r04tree; else d=.; fi
    (cd $d && timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --diff-reps 0) > gpurun_out/${tag}_e2e_$t.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_e2e_$t.json'));e=d['e2e'];print('$t',e['runs_per_s'],e['total_s'],e['ingest_only_s'],e['ingest_gb_per_s'],e['device_and_handover_s'])"
  done ;;
esac
case "$1" in
bisect3)
  for b in bench.py bench_prev.py bench.py; do
    timeout -k 10 300 python -u $b --no-cpu-baseline --e2e-runs 0 --diff-reps 0 > gpurun_out/${tag}_x.json 2>gpurun_out/${tag}_x.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_x.json'));print('$b',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['frac'],str(d.get('step_host_ms_rank0'))[:40])"
  done ;;
esac
case "$1" in
c5k)
  timeout -k 10 500 python -u bench.py --config c5 --runs-total 1000 --steps 2 --warmup 1 --e2e-runs 0 --no-cpu-baseline > gpurun_out/${tag}_c5k.json 2> gpurun_out/${tag}_c5k.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${tag}_c5k.json'));print('parts4',d['value'],d['ms_per_step'],d['pass_phases_rank0'])"
  timeout -k 10 500 python -u bench.py --config c5 --runs-total 1000 --steps 2 --warmup 1 --e2e-runs 0 --no-cpu-baseline --set load_parts=1 > gpurun_out/${tag}_c5k1.json 2> gpurun_out/${tag}_c5k1.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${tag}_c5k1.json'));print('parts1',d['value'],d['ms_per_step'],d['pass_phases_rank0'])" ;;
esac
case "$1" in
fuse)  # k_build's marksimp tail: its tests, then the C3 line with the tail on / off / on
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "build_marksimp or holds_before or build_tiers or heavy_indegree or repeated_passes or synthetic_corpus" > gpurun_out/${tag}_fuse_t.log 2>&1
  rc=$?; tail -2 gpurun_out/${tag}_fuse_t.log; [ $rc -eq 0 ] || exit $rc
  for v in 1 0 1; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-runs 0 --diff-reps 0 --set build_marksimp=$v > gpurun_out/${tag}_fuse$v.json 2> gpurun_out/${tag}_fuse$v.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_fuse$v.json'));print('ms_fuse $v',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['frac'],d['roofline'].get('avg_launch_ms'))"
  done ;;
esac
case "$1" in
loadab)  # one C5 batch's load: upload parts 4 vs 1, then a kernel + copy trace of parts 4
  timeout -k 10 300 python -u tools/load_probe.py 143 load_parts=4 > gpurun_out/${tag}_lp4.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/load_probe.py 143 load_parts=1 > gpurun_out/${tag}_lp1.log 2>&1 || exit 1
  tail -2 gpurun_out/${tag}_lp4.log; tail -2 gpurun_out/${tag}_lp1.log
  cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${tag}_lptrace -o lp -- python3 $GRAFT_REPO_ROOT/tools/load_probe.py 143 load_parts=4 > $GRAFT_REPO_ROOT/gpurun_out/${tag}_lptrace.log 2>&1 || exit 1
  tail -2 $GRAFT_REPO_ROOT/gpurun_out/${tag}_lptrace.log ;;
esac
case "$1" in
loaddbg)  # load phases of one C5 batch and of the 1k-run batched pass (NEMO_LOAD_DEBUG)
  NEMO_LOAD_DEBUG=1 timeout -k 10 300 python -u tools/load_probe.py 143 load_parts=4 > gpurun_out/${tag}_lpdbg.log 2>&1 || exit 1
  tail -8 gpurun_out/${tag}_lpdbg.log
  NEMO_LOAD_DEBUG=1 timeout -k 10 500 python -u bench.py --config c5 --runs-total 1000 --steps 2 --warmup 1 --e2e-runs 0 --no-cpu-baseline > gpurun_out/${tag}_c5kdbg.json 2> gpurun_out/${tag}_c5kdbg.err || exit 1
  grep nemo_load gpurun_out/${tag}_c5kdbg.err | tail -14
  python -c "import json;d=json.load(open('gpurun_out/${tag}_c5kdbg.json'));print(d['value'],d['ms_per_step'],d['pass_phases_rank0'])" ;;
esac
case "$1" in
parts)  # interleaved part uploads: the big-graph tests, then the C5 1k line with parts 4 / 1
  timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_batched.py tests/test_gpu_c5_shape.py tests/test_gpu_deep.py tests/test_gpu_scale.py > gpurun_out/${tag}_t.log 2>&1
  rc=$?; tail -2 gpurun_out/${tag}_t.log; [ $rc -eq 0 ] || exit $rc
  NEMO_LOAD_DEBUG=1 timeout -k 10 300 python -u tools/load_probe.py 143 > gpurun_out/${tag}_lpdbg.log 2>&1 || exit 1
  tail -4 gpurun_out/${tag}_lpdbg.log
  for v in 4 1; do
    NEMO_LOAD_DEBUG=1 timeout -k 10 500 python -u bench.py --config c5 --runs-total 1000 --steps 2 --warmup 1 --e2e-runs 0 --no-cpu-baseline --set load_parts=$v > gpurun_out/${tag}_c5k$v.json 2> gpurun_out/${tag}_c5k$v.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_c5k$v.json'));print('parts $v',d['value'],d['ms_per_step'],d['pass_phases_rank0'])"
  done ;;
esac
case "$1" in
c5kdbg)
  NEMO_LOAD_DEBUG=1 timeout -k 10 500 python -u bench.py --config c5 --runs-total 1000 --steps 2 --warmup 1 --e2e-runs 0 --no-cpu-baseline > gpurun_out/${tag}_c5k.json 2> gpurun_out/${tag}_c5k.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${tag}_c5k.json'));print(d['value'],d['ms_per_step'],d['pass_phases_rank0'])"
  grep -E "dalloc|release" gpurun_out/${tag}_c5k.err | tail -40 ;;
esac
case "$1" in
prefetch)  # batched passes with prefetch + parts: tests, then the C5 1k line and the C3 line
  timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_batched.py tests/test_gpu_c5_shape.py tests/test_gpu_diff.py > gpurun_out/${tag}_t.log 2>&1
  rc=$?; tail -2 gpurun_out/${tag}_t.log; [ $rc -eq 0 ] || exit $rc
  NEMO_LOAD_DEBUG=1 timeout -k 10 500 python -u bench.py --config c5 --runs-total 1000 --steps 2 --warmup 1 --e2e-runs 0 --no-cpu-baseline > gpurun_out/${tag}_c5k.json 2> gpurun_out/${tag}_c5k.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${tag}_c5k.json'));print(d['value'],d['ms_per_step'],d['pass_phases_rank0'])"
  grep -E "dalloc" gpurun_out/${tag}_c5k.err | tail -8
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-runs 0 --diff-reps 0 > gpurun_out/${tag}_c3.json 2> gpurun_out/${tag}_c3.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${tag}_c3.json'));print('c3',d['value'],d['ms_per_step'],d['roofline']['frac'])" ;;
esac
case "$1" in
async)  # load_async: its tests, then the C5 1k line
  timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_batched.py tests/test_gpu_c5_shape.py "tests/test_gpu_parity.py::test_load_async_reports_at_mark" "tests/test_gpu_parity.py::test_cycle_refused" > gpurun_out/${tag}_t.log 2>&1
  rc=$?; tail -2 gpurun_out/${tag}_t.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 500 python -u bench.py --config c5 --runs-total 1000 --steps 2 --warmup 1 --e2e-runs 0 --no-cpu-baseline > gpurun_out/${tag}_c5k.json 2> gpurun_out/${tag}_c5k.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${tag}_c5k.json'));print(d['value'],d['ms_per_step'],d['pass_phases_rank0'])" ;;
esac
case "$1" in
relax)  # k_build's relaxation levels: parity (tiers, C3 full, deep, batched), then the C3 line relax on / off / on
  timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_golden.py tests/test_gpu_deep.py > gpurun_out/${tag}_t.log 2>&1
  rc=$?; tail -2 gpurun_out/${tag}_t.log; [ $rc -eq 0 ] || exit $rc
  for v in 1 0 1; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-runs 0 --diff-reps 0 --set build_relax=$v > gpurun_out/${tag}_c3_$v.json 2> gpurun_out/${tag}_c3_$v.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_c3_$v.json'));print('relax $v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac'])"
  done ;;
esac
case "$1" in
c5kab)  # C5 1k line: load_parts 8 and 125-run batches against the defaults
  for args in "" "--set load_parts=8" "--batch-runs 125"; do
    timeout -k 10 500 python -u bench.py --config c5 --runs-total 1000 --steps 2 --warmup 1 --e2e-runs 0 --no-cpu-baseline $args > gpurun_out/${tag}_x.json 2> gpurun_out/${tag}_x.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_x.json'));print('[$args]',d['value'],d['ms_per_step'],d['pass_phases_rank0'])"
  done ;;
esac
case "$1" in
c5kbs)  # C5 1k line: smaller batches
  for b in 112 100 84; do
    timeout -k 10 500 python -u bench.py --config c5 --runs-total 1000 --steps 2 --warmup 1 --e2e-runs 0 --no-cpu-baseline --batch-runs $b > gpurun_out/${tag}_x.json 2> gpurun_out/${tag}_x.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${tag}_x.json'));print('[$b]',d['value'],d['ms_per_step'],d['config']['batch_sizes'][:2],d['pass_phases_rank0']['load_s'][:3],d['pass_phases_rank0']['analyse_s'][:3])"
  done ;;
esac
case "$1" in
diffat)  # where the step issues the diff: after mark / after the protos, both diff modes
  for m in reference per_run; do
    for at in mark protos mark protos; do
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-runs 0 --diff-reps 0 --diff-mode $m --diff-at $at > gpurun_out/${tag}_x.json 2> gpurun_out/${tag}_x.err || exit 1
      python -c "import json;d=json.load(open('gpurun_out/${tag}_x.json'));print('$m $at',d['value'],d['ms_per_step'])"
    done
  done ;;
esac
