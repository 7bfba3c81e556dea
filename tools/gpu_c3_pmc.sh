# PMC of the x6 conv3 variants (build/w6n = -DICLR17_C3N_W6=1): in isolation (tools/c3_epi_time.py,
# B=32 / 64) and inside the training step (ICLR17_TRAIN_W6=0 / 1): L2 hit rate, SQ issue / wait counters
set -u
O=gpurun_out/c3_pmc; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
R=$GRAFT_REPO_ROOT
export ICLR17_LIB=$R/build/w6n/libiclr17.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run -- python3 $R/tools/c3_epi_time.py --rounds 10 > $R/$O/trace.log 2>&1 || { tail $R/$O/trace.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d $R/$O/p1 -o run -- python3 $R/tools/c3_epi_time.py --rounds 10 > $R/$O/p1.log 2>&1 || { tail $R/$O/p1.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $R/$O/p2 -o run -- python3 $R/tools/c3_epi_time.py --rounds 10 > $R/$O/p2.log 2>&1 || { tail $R/$O/p2.log; exit 1; }
for v in 0 1; do
ICLR17_TRAIN_W6=$v timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d $R/$O/t1_$v -o run -- python3 $R/bench.py --mode train --batch 32 --no-cpu-baseline --steps 5 --warmup 2 > $R/$O/t1_$v.log 2>&1 || { tail $R/$O/t1_$v.log; exit 1; }
ICLR17_TRAIN_W6=$v timeout -s KILL 180 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $R/$O/t2_$v -o run -- python3 $R/bench.py --mode train --batch 32 --no-cpu-baseline --steps 5 --warmup 2 > $R/$O/t2_$v.log 2>&1 || { tail $R/$O/t2_$v.log; exit 1; }
done
echo done
