#!/bin/bash
# Sharded device loop before/after, one GPU box:
#   gpurun -- bash scripts/gpu_dsp.sh TAG [TREE_OLD]
# 1. the sharded / device-sampler GPU tests of this tree;
# 2. scripts/ds_shard_profile.py under rocprofv3 --kernel-trace --stats for
#    this tree and (optionally) an older build's worktree, at the C4 rank
#    shape (W = 65 536 over 8 gloo ranks = 8 192 walkers a rank) and at
#    W = 16 384 over 2 ranks.  Output: gpurun_out/dsp_TAG/.
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
run() {  # name tree R W
  local name=$1 tree=$2 R=$3 W=$4
  HB_TREE=$tree timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name/%pid%" -o run -- \
    python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$R" --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) "$ROOT/scripts/ds_shard_profile.py" "$OUT/$name.json" "$W" 100 20 \
    > "$OUT/$name.log" 2>&1 || { tail -30 "$OUT/$name.log"; return 1; }
  tail -1 "$OUT/$name.log"
}
run new_r8 "$ROOT" 8 65536 && run new_r2 "$ROOT" 2 16384 || exit 1
if [ -n "$OLD" ]; then
  run old_r8 "$ROOT/$OLD" 8 65536 && run old_r2 "$ROOT/$OLD" 2 16384 || exit 1
fi
python3 "$ROOT/scripts/dsp_summary.py" "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
