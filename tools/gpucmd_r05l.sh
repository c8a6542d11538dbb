#!/bin/bash
# Round 5, call L: the full GPU suite and smoke() at the final kernels (profiles/r05_gpu_tests.txt).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
tail -3 $O/gpu_tests.txt
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/gpu_tests.txt | head -40; exit 1; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
