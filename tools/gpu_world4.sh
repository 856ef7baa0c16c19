#!/bin/bash
# smoke(), then the N-rank rehearsal at world 4 on one GPU through bench.py's launcher and through torch.distributed.run
set -o pipefail
OUT=gpurun_out/w4
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" && \
QCART_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 4 --batch 16384 --steps 3 --warmup 1 \
    --no-cpu-baseline --digest-envs 16384 --launch-timeout 360 > $OUT/launcher4.json 2> $OUT/launcher4.err && \
QCART_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --batch 16384 --steps 3 --warmup 1 \
    --no-cpu-baseline --digest-envs 16384 > $OUT/torchrun4.json 2> $OUT/torchrun4.err && \
timeout -k 10 400 python bench.py --batch 65536 --steps 3 --warmup 1 --no-cpu-baseline --digest-envs 16384 \
    > $OUT/whole1.json 2> $OUT/whole1.err && \
python - <<'PY'
import json
r = {k: json.loads([l for l in open(f"gpurun_out/w4/{k}.json") if l.startswith("{")][-1]) for k in ("launcher4", "torchrun4", "whole1")}
for k, v in r.items():
    print(k, v["n_gpus"], v["config"]["world_size_seen"], v["config"]["global_batch"], v["config"]["rccl"] and v["config"]["rccl"]["gathered_envs"], "%.3e" % v["value"], v["psi_digests"])
print("digests equal:", r["launcher4"]["psi_digests"] == r["whole1"]["psi_digests"] == r["torchrun4"]["psi_digests"])
PY
