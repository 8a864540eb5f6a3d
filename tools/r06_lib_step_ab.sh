# config-2 step A/B between libraries (LIBS), interleaved in separate processes
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06i}
LIBS=${LIBS:-"libvp_hip"}
mkdir -p $O
for i in 1 2 3; do
  for L in $LIBS; do
    VP_HIP_LIB=videopainter_amd/_lib/$L.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_${L}_$i.log 2>&1 || exit 1
    echo "$i $L $(grep -o '"value": [0-9.]*' $O/bench_${L}_$i.log) $(grep -o '"gemm": {[^}]*' $O/bench_${L}_$i.log | grep -o '"achieved": [0-9.]*')"
  done
done
