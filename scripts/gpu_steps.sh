#!/bin/bash
# Generic GPU session: runs "name timeout cmd..." steps given as lines on
# stdin-free arguments file ($1), each under its own time limit, output in
# gpurun_out/<name>.log; stops at the first fault-like exit status (> 1, e.g.
# 124/134/137/139) without starting further GPU work.
mkdir -p gpurun_out
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 4 "gpurun_out/$name.log" | cut -c1-2000
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
while read -r name to rest; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue;; esac
  eval "step $name $to $rest"
done < "$1"
