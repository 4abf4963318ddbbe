set -u
export TMPDIR=/tmp
O=gpurun_out/p; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do timeout -k 10 300 python bench.py --steps 40 --warmup 5 --cpu-baseline 0 --profile-steps 0 > $O/b$r.json 2>/dev/null || exit 1; python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $O/b$r.json; done
