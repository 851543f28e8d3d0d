cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/b20
for k in 1 2 3; do
  timeout -k 10 250 python3 bench.py --steps 20 --warmup 5 --no-sharded --no-neumf --no-eval --no-large --no-cpu-baseline > gpurun_out/b20/b20_$k.json 2> gpurun_out/b20/b20_$k.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/b20/b20_$k.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d.get('stream_recoveries'), d['step_errors'])"
done
