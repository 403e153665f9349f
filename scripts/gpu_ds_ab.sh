#!/bin/bash
# Interleaved A/B of the device-resident loop (W = 4096, N = 1024) over
# library variants and environment knobs, on one GPU box:
#   gpurun -- bash scripts/gpu_ds_ab.sh TAG ROUNDS "name=ENV[,ENV] name=..."
# ENV items: HBMI_LIB=<path> (a lib/variants build) or any HB_DS_* knob; "base"
# with no '=' runs the default library.  Prints ms/iteration per run and the
# logLmap / counters (identical across variants that only move work around).
set -o pipefail
TAG=${1:-x}
ROUNDS=${2:-2}
VARS=${3:-base}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/dsab_$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
for r in $(seq 1 "$ROUNDS"); do
  for v in $VARS; do
    name=${v%%=*}
    envs=""
    [ "$v" != "$name" ] && envs=$(echo "${v#*=}" | tr ',' ' ')
    [ -n "$envs" ] && envs=$(echo "$envs" | sed "s|HBMI_LIB=|HBMI_LIB=$ROOT/|g")
    env $envs timeout -k 10 120 python3 scripts/sampler_rate.py --device --iters 320 > "$OUT/${name}_$r.json" 2> "$OUT/${name}_$r.err" \
      || { tail -5 "$OUT/${name}_$r.err"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], round(d['ms_per_iter'],4), d['logLmap'], d['stats']['nswap'], d['stats']['cold_acc'])" \
      "$OUT/${name}_$r.json" "$name" "$r"
  done
done
