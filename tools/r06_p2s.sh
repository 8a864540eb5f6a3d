# p2s (16x16x32 p2 pipeline): parity tests, then interleaved clock A/B against p2a, then the step A/B
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06c}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "p2s or attn_p2a" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  VP_HIP_LIB=videopainter_amd/_lib/libvp_hip_clk.so timeout -k 10 200 python tools/attn_clock.py --variants p2a,p2s --label r$i >> $O/clock_ab.log 2>&1 || exit 2
done
grep '^r' $O/clock_ab.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_p2a_$i.log 2>&1 || exit 3
  VP_ATTN_UNBOUNDED_MODE=p2s VP_ATTN_BOUNDED_MODE=p2s timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_p2s_$i.log 2>&1 || exit 4
done
for f in $O/bench_*.log; do echo $f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"attention": {[^}]*' $f | head -c 200); done
