set -o pipefail
# per-instance regression table (scripts/regress.py), the round-4 local-DFS knobs undone one
# at a time on ta021 (which one cost 9.26 -> 9.71 s?), and a PMC pass on ta021's front kernel
out=gpurun_out/r5reg; mkdir -p $out
timeout -k 10 240 python -u scripts/regress.py > $out/table_default.txt 2>&1 || { tail -20 $out/table_default.txt; exit 1; }
grep -v amdgpu.ids $out/table_default.txt
for v in "TTS_LOCAL_STRIDE=0" "TTS_LOCAL_WIDE_STEPS=4" "TTS_LOCAL_NARROW_STEPS=4" "TTS_LOCAL_STRIDE=0 TTS_LOCAL_WIDE_STEPS=4 TTS_LOCAL_NARROW_STEPS=4"; do
  tag=$(echo $v | tr ' =' '_-')
  env $v timeout -k 10 120 python -u scripts/regress.py 21:0 > $out/ta021_$tag.txt 2>&1 || { tail -20 $out/ta021_$tag.txt; exit 1; }
  echo "== $v"; grep ta021 $out/ta021_$tag.txt
done
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $out/pmc021a -o run -- python3 scripts/profile_workload.py ta021 > $out/pmc021a.log 2>&1 || { tail -20 $out/pmc021a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE -d $out/pmc021b -o run -- python3 scripts/profile_workload.py ta021 > $out/pmc021b.log 2>&1 || { tail -20 $out/pmc021b.log; exit 1; }
python3 scripts/pmc_summary.py $out/pmc021a pfsp_front > $out/pmc021_summary.txt && python3 scripts/pmc_summary.py $out/pmc021b pfsp_front >> $out/pmc021_summary.txt && cat $out/pmc021_summary.txt
