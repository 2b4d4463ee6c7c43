# sourced by tools/gpu_*.sh: run a GPU step under its own time limit; a test failure (rc 1) is reported and the
# script goes on, anything that looks like a fault, abort, kill or time limit ends the script
step() {
  local secs=$1; shift
  timeout -k 10 "$secs" "$@"
  local rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then
    echo "step failed hard (rc $rc): $*" >&2
    exit $rc
  fi
  [ $rc -ne 0 ] && echo "step rc $rc: $*" >&2
  return 0
}
