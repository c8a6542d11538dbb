#!/bin/bash
# Round 6, call I: the whole GPU suite (no -x: every failure listed) and smoke() after
# the macro cleanup; the C3 leg's profile-instance check is expected to fail until the
# leg is re-profiled at the new split instance.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
tail -3 $O/gpu_tests.txt
grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
exit $rc
