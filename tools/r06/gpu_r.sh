#!/bin/bash
# Round 6, call R: the whole GPU suite + smoke() at the final sources.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
tail -3 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
