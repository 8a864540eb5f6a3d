# round-6 final HEAD, part 2 (benches): the driver's default line, config 5 / config 2 under rocprof, training, config 4
set -u
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || exit 1
echo bench $(grep -o '"value": [0-9.]*' $O/bench.log | head -1)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5line.log 2>&1 || exit 2
echo c5 $(grep -o '"value": [0-9.]*' $O/c5line.log)
timeout -k 10 300 python tools/bench_train.py --steps 6 --warmup 2 > $O/train.log 2>&1 || exit 3
tail -1 $O/train.log | cut -c1-200
timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4line.log 2>&1 || exit 4
echo c4 $(grep -o '"value": [0-9.]*' $O/c4line.log)
