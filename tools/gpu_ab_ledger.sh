set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_bench.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pt.log 2>&1 || { tail -30 $OUT/pt.log; exit 1; }
tail -2 $OUT/pt.log
timeout -k 10 300 python bench.py > $OUT/b_timed.json 2> $OUT/b_timed.err || exit 1
timeout -k 10 300 python bench.py --no-timed-ledger --no-cpu-baseline --no-in-solver > $OUT/b_untimed.json 2> $OUT/b_untimed.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-in-solver > $OUT/b_timed2.json 2> $OUT/b_timed2.err || exit 1
rm -rf $OUT/prof2
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-in-solver --no-small > $OUT/b_rocprof.json 2> $OUT/b_rocprof.err || exit 1
echo done
