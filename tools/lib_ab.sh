# same-box A/B of two library builds at one config: tools/lib_ab.sh <config> <old.so> <out>
set -o pipefail
C=$1; OLD=$2; O=$3; : > $O
F="--config $C --steps 200 --warmup 50 --cpu-baseline 0 --collate-bench 0 --infer-bench 0 --profile-steps 0"
for r in 1 2 3; do
 for v in old new; do
  if [ $v = old ]; then L=$OLD; else L=cgr-mpnn-3d_amd/cgr_mpnn_3D/_amd/lib/libcgr_mpnn3d.so; fi
  val=$(CGR_MPNN3D_LIB=$PWD/$L timeout -k 10 120 python bench.py $F 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'])") || exit 1
  echo "$r $v $val" | tee -a $O
 done
done
