#!/bin/bash
# two-rank rehearsal of bench.py's N > 1 path on one GPU (gloo exchange, both ranks on GPU 0)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
MBLS_BENCH_SAME_DEVICE=1 MBLS_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 6 --warmup 2 --no-cpu --no-mix --msm-total-log 21 \
  > gpurun_out/r4h_rehearsal.json 2> gpurun_out/r4h_rehearsal.err || { tail -30 gpurun_out/r4h_rehearsal.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r4h_rehearsal.json').read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], d['msm_step_ms'], d['config4_msm_sharded']['result_digest'])"
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu --no-mix --msm-total-log 21 > gpurun_out/r4h_n1.json 2> gpurun_out/r4h_n1.err || { tail -20 gpurun_out/r4h_n1.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4h_n1.json')); print(d['value'], d['n_gpus'], d['config4_msm_sharded']['result_digest'], d['mix_g2msm_batched_ntt'] if 'mix_g2msm_batched_ntt' in d else '')"
