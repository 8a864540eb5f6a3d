#!/bin/bash
# round 3: 2-rank gloo rehearsals of the multi-rank bench paths on the one GPU of the box (functional: both ranks on
# cuda:0), default --bcast (scatter_allgather: P2P scatter + all_gather_into_tensor, host-staged on gloo)
set -u
export TMPDIR=/tmp VP_BENCH_DIST_BACKEND=gloo
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
run r03_rehearsal_dp2_gloo_1gpu 400 $TR --master-port 29511 bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline
run r03_rehearsal_cfgpair2_gloo_1gpu 400 $TR --master-port 29512 bench.py --gpus 2 --steps 1 --warmup 1 --mode cfgpair --no-cpu-baseline
run r03_rehearsal_stages2_gloo_1gpu 500 $TR --master-port 29513 bench.py --gpus 2 --steps 1 --warmup 0 --mode stages --no-cpu-baseline
exit 0
