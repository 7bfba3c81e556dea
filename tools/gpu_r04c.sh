set -u
O=gpurun_out/r04c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python tools/x6k_time.py > $O/time.log 2>&1 || { cat $O/time.log; exit 1; }
cat $O/time.log
REPS=3 TOOL=tools/x6k_time.py OUT_NAME=r04c/pmc timeout -k 10 400 bash tools/pmc_kernel.sh > $O/pmc_run.log 2>&1 || { tail $O/pmc_run.log; exit 1; }
python tools/pmc_csv_summary.py $O/pmc > $O/pmc_summary.txt; cat $O/pmc_summary.txt
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('x6', d['value'], {k: v['ms'] for k, v in d['layers'].items()}); b=d['bf16_mode']; print('bf16', b['value'], {k: v['ms'] for k, v in b['layers'].items()})" $O/bench.json
