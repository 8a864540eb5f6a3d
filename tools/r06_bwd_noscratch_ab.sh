set -u
# dK / dV tile body on recomputed lane offsets (VP_DKDV_OPQ=1, default) against the spilled kernel-wide offsets
# (libvp_hip_bwdold.so = the same sources built with -DVP_DKDV_OPQ=0): interleaved attention backward, then training.
mkdir -p gpurun_out/r06bw
for i in 1 2 3 4; do
  timeout -k 10 100 python tools/bench_attn_bwd.py --iters 10 >> gpurun_out/r06bw/new.log 2>&1 || exit 2
  VP_HIP_LIB=videopainter_amd/_lib/libvp_hip_bwdold.so timeout -k 10 100 python tools/bench_attn_bwd.py --iters 10 >> gpurun_out/r06bw/old.log 2>&1 || exit 3
done
echo new; grep -o '"bwd_ms": [0-9.]*' gpurun_out/r06bw/new.log; echo old; grep -o '"bwd_ms": [0-9.]*' gpurun_out/r06bw/old.log
for i in 1 2; do
  timeout -k 10 200 python tools/bench_train.py --steps 6 --warmup 2 >> gpurun_out/r06bw/train_new.log 2>&1 || exit 4
  VP_HIP_LIB=videopainter_amd/_lib/libvp_hip_bwdold.so timeout -k 10 200 python tools/bench_train.py --steps 6 --warmup 2 >> gpurun_out/r06bw/train_old.log 2>&1 || exit 5
done
echo train_new; grep -o '"value": [0-9.]*' gpurun_out/r06bw/train_new.log; echo train_old; grep -o '"value": [0-9.]*' gpurun_out/r06bw/train_old.log
