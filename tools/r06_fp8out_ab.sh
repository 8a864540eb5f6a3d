set -u
# config 5 with the attention output projection in fp8 (default) against bf16 (--fp8-out-bf16), interleaved
mkdir -p gpurun_out/r06fo
for i in 1 2; do
  timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06fo/new$i.log 2>&1 || exit 2
  echo new $(grep -o '"value": [0-9.]*' gpurun_out/r06fo/new$i.log | head -1)
  timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --fp8-out-bf16 > gpurun_out/r06fo/old$i.log 2>&1 || exit 3
  echo old $(grep -o '"value": [0-9.]*' gpurun_out/r06fo/old$i.log | head -1)
done
grep -h "rel-L2" gpurun_out/r06fo/new1.log gpurun_out/r06fo/old1.log
