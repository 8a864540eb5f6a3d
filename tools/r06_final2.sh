# round-6 HEAD measurements after the grid-tail / persistent-attention work: config 5 under rocprof, config 2 under
# rocprof, the training step, the attention's PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes)
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06h}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5line.log 2>&1 || exit 1
echo c5 $(grep -o '"value": [0-9.]*' $O/c5line.log)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/c2prof.log 2>&1 || exit 2
echo c2prof $(grep -o '"value": [0-9.]*' $O/c2prof.log)
timeout -k 10 400 python tools/bench_train.py --steps 6 --warmup 2 > $O/train.log 2>&1 || exit 3
tail -1 $O/train.log | cut -c1-200
timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4line.log 2>&1 || exit 4
echo c4 $(grep -o '"value": [0-9.]*' $O/c4line.log)
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/pmc_attention_$C -o k --output-format csv -- python tools/bench_kernels.py --only attention --iters 2 --variant p2a > $O/pmc_attention_$C.log 2>&1 || exit 5
done
echo traffic done
