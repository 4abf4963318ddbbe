# A/B of the NT kernels' per-k-step accumulation (CGR_B3_STEP_ACC): the in-tree library against
# abvar/base (built with -DCGR_B3_STEP_ACC=0), cfg2, 3 alternating runs each; plus the
# learnable-skip precision diagnostic on the in-tree library.
set -e
mkdir -p gpurun_out/stepacc
timeout -k 10 300 python tools/diag/cfg_err.py > gpurun_out/stepacc/cfg_err_new.txt 2>&1
for i in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export CGR_MPNN3D_LIB=$PWD/abvar/base/libcgr_mpnn3d.so; else unset CGR_MPNN3D_LIB; fi
    timeout -k 10 200 python bench.py --config ${CFG:-cfg2} --steps 100 --warmup 30 --cpu-baseline 0 --collate-bench 0 --infer-bench 0 --profile-steps 0 > gpurun_out/stepacc/${CFG:-cfg2}_${v}_$i.json 2>/dev/null
  done
done
unset CGR_MPNN3D_LIB
