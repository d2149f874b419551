cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/profq_lvl; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAVES -d $OUT/p1 -o p1 --output-format csv -- python tools/prof_frames.py --frames 3 > $OUT/p1.log 2>&1
