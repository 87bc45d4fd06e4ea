# Round 6: is the interleave's loss the unstaged y stores?  contiguous ranges with / without LDS-staged y
# writes (VBC_SLOT_STAGE=0) against the interleave (which stores each chunk when it ends)
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab.py --workload fe --dtype f64 --graph --reps 20 --rounds 5 --copies 2 --variants "VBC_SLOT_ILV=0;VBC_SLOT_ILV=0,VBC_SLOT_STAGE=0;VBC_SLOT_ILV=1" > gpurun_out/r06s_fe_stage.log 2>&1 || { tail -20 gpurun_out/r06s_fe_stage.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06s_fe_stage.log | tail -6
