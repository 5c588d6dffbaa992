#!/bin/bash
# round-2 GPU check: new tests, default bench line, in-process group and
# 2-rank torchrun rehearsal on one GPU.  usage: tools/gpu_r2.sh OUTDIR [tests...]
set -o pipefail
OUT=${1:-gpurun_out/r2}; shift
mkdir -p $OUT
T=${@:-tests}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --devices 0,0 --steps 10 > $OUT/group2.json 2> $OUT/group2.err || { echo "group failed"; tail -20 $OUT/group2.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --devices 0,0 --steps 10 --no-cpu > $OUT/ranks2.json 2> $OUT/ranks2.err || { echo "ranks failed"; tail -20 $OUT/ranks2.err; exit 1; }
echo done
