set -u
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
for lib in clk clk_l2 clk clk_l2; do
  VP_HIP_LIB=videopainter_amd/_lib/libvp_hip_$lib.so timeout -k 10 200 python tools/attn_clock.py --variants p2a --label $lib --dump $O/stamps_$lib >> $O/clock_ab.log 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $O/pmc_l2 -o k --output-format csv -- python tools/bench_kernels.py --only attention --iters 2 --variant p2a > $O/pmc_l2.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum --kernel-trace -d $O/pmc_l2b -o k --output-format csv -- python tools/bench_kernels.py --only attention --iters 2 --variant p2a > $O/pmc_l2b.log 2>&1 || exit 3
echo done
