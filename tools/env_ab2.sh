set -o pipefail
# Same-box A/B of runtime knobs (no rebuild): hardware queues per process (default 4 on the box)
O=gpurun_out/r06_env_ab.txt; : > $O
F="--steps 200 --warmup 50 --cpu-baseline 0 --collate-bench 0 --infer-bench 0 --profile-steps 0"
for r in 1 2 3; do
 for v in base q2 q8; do
  case $v in base) E="";; q2) E="GPU_MAX_HW_QUEUES=2";; q8) E="GPU_MAX_HW_QUEUES=8";; esac
  val=$(env $E timeout -k 10 120 python bench.py $F 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'])") || exit 1
  echo "$r $v $val" | tee -a $O
 done
done
