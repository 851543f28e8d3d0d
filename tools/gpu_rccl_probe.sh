# RCCL capture probes (r04 + r05), one process per probe under its own time
# limit; every probe's exit status is printed, and the script exits with the
# first non-zero one (a hang shows as 124 / 137).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/rccl_probe
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 90 python3 "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(grep -v amdgpu.ids $OUT/$name.log | grep -v '^ *$' | tail -3 | tr '\n' ' ')"
  return $rc
}
run a2a_del_destroy tools/rccl_capture_probe.py all_to_all del_destroy &&
run a2a_exit tools/rccl_capture_probe.py all_to_all exit &&
run ag_destroy tools/rccl_capture_probe.py all_gather destroy &&
run sharded_with_destroy tools/rccl_capture_probe.py sharded with_destroy &&
run sharded_del_destroy tools/rccl_capture_probe.py sharded del_destroy &&
run sharded_exit tools/rccl_capture_probe.py sharded exit
rc=$?
echo "probes rc=$rc"
exit $rc
