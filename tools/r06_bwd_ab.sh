# attention backward A/B over libraries (LIBS), interleaved, then rocprof per-kernel stats for each
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06f}
LIBS=${LIBS:-"libvp_hip libvp_hip_bwdnoslp"}
mkdir -p $O
for i in 1 2 3; do
  for L in $LIBS; do
    VP_HIP_LIB=videopainter_amd/_lib/$L.so timeout -k 10 200 python tools/bench_attn_bwd.py --iters 10 >> $O/ab_$L.log 2>&1 || exit 1
    echo "$i $L $(tail -1 $O/ab_$L.log | cut -c1-120)"
  done
done
for L in $LIBS; do
  VP_HIP_LIB=videopainter_amd/_lib/$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$L -o b --output-format csv -- python tools/bench_attn_bwd.py --iters 10 > $O/prof_$L.log 2>&1 || exit 2
  echo $L; grep bwd_ $O/prof_$L/b_kernel_stats.csv | cut -d, -f1-4
done
