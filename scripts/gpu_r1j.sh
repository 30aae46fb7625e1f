#!/bin/bash
o=gpurun_out/r1j; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 &&
timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $o/n1.json 2> $o/n1.err &&
timeout -k 10 200 python scripts/graph_probe.py > $o/graph_probe.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- python scripts/profile_workload.py ta014 > $o/trace.log 2>&1 &&
python scripts/timeline.py $o/trace 30 > $o/timeline.txt
rc=$?
tail -2 $o/gpu_tests.log; cat $o/n1.json; grep "poll=1" $o/graph_probe.txt; cat $o/timeline.txt
exit $rc
