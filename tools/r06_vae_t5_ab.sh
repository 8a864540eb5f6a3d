set -u
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
for i in 1 2; do
  for L in libvp_hip libvp_hip_vaenoslp; do
    VP_HIP_LIB=videopainter_amd/_lib/$L.so timeout -k 10 300 python tools/bench_vae.py --iters 2 > $O/vae_${L}_$i.log 2>&1 || exit 1
    echo "$i $L $(tail -1 $O/vae_${L}_$i.log | cut -c1-250)"
    VP_HIP_LIB=videopainter_amd/_lib/$L.so timeout -k 10 300 python tools/bench_t5.py > $O/t5_${L}_$i.log 2>&1 || exit 2
    echo "$i $L $(tail -1 $O/t5_${L}_$i.log | cut -c1-200)"
  done
done
