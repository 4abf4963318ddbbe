set -o pipefail
O=gpurun_out/r05_s3_env_ab.txt; : > $O
F="--steps 200 --warmup 50 --cpu-baseline 0 --collate-bench 0 --infer-bench 0 --profile-steps 0"
for r in 1 2 3; do
 for v in base devkernarg prepsplit; do
  case $v in base) E="";; devkernarg) E="HIP_FORCE_DEV_KERNARG=1";; prepsplit) E="CGR_PREP_SPLIT=1";; esac
  val=$(env $E timeout -k 10 120 python bench.py $F 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'])") || exit 1
  echo "$r $v $val" | tee -a $O
 done
done
