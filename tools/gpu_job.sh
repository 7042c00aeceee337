#!/bin/bash
# One parametrized GPU-box runner (replaces the round-2 single-use gpu_s*.sh scripts).
# Each argument is one step "KIND [ARGS...]" (quoted); steps run in order, each under its own time
# limit, and the job stops at the first failing step (no retries; a timeout / abort / segfault ends it).
#
#   tests [PYTEST ARGS]        GPU test suite (default: all of tests/ -m gpu)
#   smoke                      __graft_entry__.smoke()
#   bench TAG [BENCH ARGS]     python bench.py ARGS -> gpurun_out/bench_TAG.log (prints the JSON head)
#   torchrun TAG N [ARGS]      bench.py under torch.distributed.run with N ranks (one-GPU rehearsal:
#                              gloo + xgmi, all ranks on GPU 0, 2 hardware queues each)
#   prof TAG [BENCH ARGS]      rocprofv3 --kernel-trace --stats of bench.py ARGS -> gpurun_out/prof_TAG,
#                              per-kernel stats (tools/kstats.py) + per-queue timeline (tools/timeline.py)
#   xgmi W [ARGS]              tools/xgmi_check.py --world W --same-device ARGS
#   ddpeq W B                  tools/ddp_equivalence.py --world W --same-device --batch B
#   ab TAG "ENV=a" "ENV=b" ... -- [BENCH ARGS]   tools/ab_multi.sh
#   py TAG SCRIPT [ARGS]       python -u SCRIPT ARGS -> gpurun_out/py_TAG.log
#   sh TAG SCRIPT [ARGS]       bash SCRIPT ARGS -> gpurun_out/sh_TAG.log (e.g. tools/pmc.sh)
#
# usage (on the box): bash tools/gpu_job.sh "tests tests/test_gpu_xgmi.py" "bench exact --gpus 1 --steps 20 --warmup 5"
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp

fatal() {   # stop the job after a timeout / abort / segfault: nothing more may touch the GPU
  case $1 in 124|134|137|139) echo "FATAL exit $1 in step '$2': stopping"; exit "$1";; esac
  [ "$1" -ne 0 ] && { echo "step '$2' failed (exit $1)"; exit "$1"; }
  return 0
}

head_json() {   # first 600 chars of the last JSON line of a log
  grep '^{' "$1" | tail -1 | cut -c1-${2:-600}
}

run_step() {
  local kind=$1; shift
  case $kind in
    tests)
      [ $# -eq 0 ] && set -- tests
      # no -x: an assertion failure (rc 1) is reported and the job goes on; a timeout, abort or
      # crash of the test process (124/134/137/139) still ends it
      timeout -k 10 1500 python -u -m pytest "$@" -m gpu -v --timeout 170 --timeout-method thread \
        > gpurun_out/tests.log 2>&1; local rc=$?
      grep -E "^(FAILED|ERROR)" gpurun_out/tests.log | head -20; tail -2 gpurun_out/tests.log
      [ $rc -eq 1 ] && { echo "tests: failures (rc 1), continuing"; return 0; }
      fatal $rc "tests $*";;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; local rc=$?
      tail -1 gpurun_out/smoke.log; fatal $rc smoke;;
    bench)
      local tag=$1; shift
      timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_$tag.log 2>&1; local rc=$?
      echo "bench $tag: $(head_json gpurun_out/bench_$tag.log)"; [ $rc -ne 0 ] && tail -20 gpurun_out/bench_$tag.log
      fatal $rc "bench $tag";;
    torchrun)
      local tag=$1 n=$2; shift 2
      MNIST_AMD_ONE_GPU=1 GPU_MAX_HW_QUEUES=2 timeout -k 10 600 python -m torch.distributed.run --standalone \
        --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node "$n" bench.py --gpus "$n" --dist-backend gloo \
        --allreduce xgmi "$@" > gpurun_out/torchrun_$tag.log 2>&1; local rc=$?
      echo "torchrun $tag: $(head_json gpurun_out/torchrun_$tag.log 900)"; [ $rc -ne 0 ] && tail -30 gpurun_out/torchrun_$tag.log
      fatal $rc "torchrun $tag";;
    prof)
      local tag=$1; shift
      local out=$R/gpurun_out/prof_$tag
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$out" -o run --output-format csv \
        -- python3 "$R/bench.py" "$@" > "$out.log" 2>&1); local rc=$?
      fatal $rc "prof $tag"
      python3 tools/kstats.py "$out" > "$out.stats.txt" 2>&1 && head -16 "$out.stats.txt"
      local csv; csv=$(find "$out" -name '*kernel_trace.csv' | head -1)
      [ -n "$csv" ] && python3 tools/timeline.py "$csv" > "$out.timeline.txt" 2>&1 && head -30 "$out.timeline.txt"
      return 0;;
    xgmi)
      local w=$1; shift
      timeout -k 10 400 python -u tools/xgmi_check.py --world "$w" --same-device "$@" > gpurun_out/xgmi_w$w.log 2>&1
      local rc=$?; tail -$((w + 2)) gpurun_out/xgmi_w$w.log; fatal $rc "xgmi $w";;
    ddpeq)
      GPU_MAX_HW_QUEUES=2 timeout -k 10 400 python -u tools/ddp_equivalence.py --world "$1" --same-device --steps 10 \
        --batch "$2" --timeout 360 > gpurun_out/ddpeq_w$1.log 2>&1; local rc=$?
      tail -3 gpurun_out/ddpeq_w$1.log; fatal $rc "ddpeq $1";;
    ab)
      bash tools/ab_multi.sh "$@"; fatal $? "ab $1";;
    py)
      local tag=$1; shift
      timeout -k 10 400 python -u "$@" > gpurun_out/py_$tag.log 2>&1; local rc=$?
      tail -40 gpurun_out/py_$tag.log; fatal $rc "py $tag";;
    sh)
      local tag=$1; shift
      timeout -k 10 900 bash "$@" > gpurun_out/sh_$tag.log 2>&1; local rc=$?
      tail -5 gpurun_out/sh_$tag.log; fatal $rc "sh $tag";;
    *)
      echo "unknown step kind '$kind'"; exit 2;;
  esac
}

for step in "$@"; do
  echo "=== $step"
  # shellcheck disable=SC2086
  eval "run_step $step"
done
echo "GPU_JOB DONE"
