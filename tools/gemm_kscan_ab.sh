set -u
for L in hip abl_nostore abl_noepi; do
  VP_HIP_LIB=videopainter_amd/_lib/libvp_$L.so timeout -k 10 200 python tools/gemm_kscan.py --iters 10 > gpurun_out/kscan_$L.log 2>&1
  rc=$?; echo "$L rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
