#!/bin/bash
# Sharded device loop before/after, one GPU box:
#   gpurun -- bash scripts/gpu_dsp.sh TAG [TREE_OLD]
# 1. the sharded / device-sampler GPU tests of this tree;
# 2. scripts/ds_shard_profile.py under rocprofv3 --kernel-trace --stats for
#    this tree and (optionally) an older build's worktree at W = 65 536 (C4's
#    ensemble): one process, 2 gloo ranks, and 8 gloo ranks (8 192 walkers a
#    rank, C4's rank shape), all sharing the box's GPU.
#    Output: gpurun_out/dsp_TAG/.
set -o pipefail
TAG=${1:-x}
OLD=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/dsp_$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_dsharded.py tests/test_dsampler.py > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
  tail -3 "$OUT/tests.log"
fi
cd /tmp && export TMPDIR=/tmp
run() {  # name tree R W [serial]
  local name=$1 tree=$2 R=$3 W=$4 mode=${5:-}
  HB_TREE=$tree timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name/%pid%" -o run -- \
    python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$R" --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) "$ROOT/scripts/ds_shard_profile.py" "$OUT/$name.json" "$W" 100 20 1024 $mode \
    > "$OUT/$name.log" 2>&1 || { tail -30 "$OUT/$name.log"; return 1; }
  tail -1 "$OUT/$name.log"
}
# concurrent ranks (wall time, host split), then ranks taking turns on the
# GPU (kernel durations of one rank alone: "s" runs)
for R in 1 2 8; do
  run new_r$R "$ROOT" $R 65536 || exit 1
  if [ -n "$OLD" ]; then run old_r$R "$ROOT/$OLD" $R 65536 || exit 1; fi
done
for R in 2 8; do
  run new_s$R "$ROOT" $R 65536 serial || exit 1
  if [ -n "$OLD" ]; then run old_s$R "$ROOT/$OLD" $R 65536 serial || exit 1; fi
done
python3 "$ROOT/scripts/dsp_summary.py" "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
