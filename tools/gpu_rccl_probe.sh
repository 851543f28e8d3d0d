# r04: which one-rank RCCL collectives survive hipGraph capture + replay, and
# whether the process group then tears down (each under its own timeout)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rccl_probe
for k in "all_to_all del_destroy" "all_to_all exit" "all_to_all del" "all_gather destroy"; do
  set -- $k
  timeout -k 10 60 python3 tools/rccl_capture_probe.py $1 $2 > gpurun_out/rccl_probe/$1_$2.log 2>&1
  rc=$?
  echo "$1 $2 rc=$rc: $(grep -v amdgpu.ids gpurun_out/rccl_probe/$1_$2.log | tail -3 | tr '\n' ' ')"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
