# quick ragged-path check: ragged GPU tests, C4 bench, C4 per-pass rocprof
export TMPDIR=/tmp; O=gpurun_out/${TAG:-r2d}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ragged or rsck or mix or sim_stream or c4 or family or batch_host" > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --mix --no-cpu > $O/mix.json 2>$O/mix.err || exit 3; cat $O/mix.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --mix > $O/prof.log 2>&1 || exit 3
cut -d, -f1-4 $O/prof_c4/run_kernel_stats.csv
