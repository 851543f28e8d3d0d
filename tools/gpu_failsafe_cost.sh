set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fs
for f in 1 0 1 0; do
  timeout -k 10 200 python3 tools/short_call.py --reps 30 --failsafe $f > gpurun_out/fs/sc_$f.json 2> gpurun_out/fs/sc_$f.err
  python3 -c "
import json,statistics as st
d=json.loads(open('gpurun_out/fs/sc_$f.json').read().strip().splitlines()[-1]); r=[x['region_us'] for x in d['reps']]
print('failsafe $f region median', st.median(r), 'min', min(r))"
done
