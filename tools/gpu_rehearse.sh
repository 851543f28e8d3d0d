# bench.py's N > 1 code path (torchrun, barrier, max-over-ranks, rank-0 JSON, the
# sharded split-step lines) rehearsed on a one-GPU box with NPROC ranks (default 2;
# at most 4 here, N = 8 is the driver's) all on cuda:0 over gloo (--rehearse-one-gpu).
# The ranks share the GPU, so a rank's k_stream may not have all of its waves
# resident: its verified calls replay a give-up on the two-kernel schedule
# (failsafe); stream_recoveries counts them.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-rehearse_n${NPROC:-2}}
mkdir -p $OUT
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus ${NPROC:-2} --steps 20 --warmup 5 --rehearse-one-gpu \
  --no-large --no-neumf --sharded-steps 4 > $OUT/bench_n.json 2> $OUT/bench_n.err
python3 -c "
import json;d=json.loads(open('$OUT/bench_n.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'value', d['value'], 'step_errors', d['step_errors'], 'recoveries', d.get('stream_recoveries'), 'parallelism', d['config']['parallelism'])
for k, v in d.get('sharded', {}).items(): print(k, v.get('n_gpus'), v.get('value'), v.get('config', {}).get('parallelism'))"
