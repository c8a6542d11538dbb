#!/bin/bash
# Round 3: PRIMAL read-ahead loop (r03t) then the shipped C2 split parity + profile (r03s).
set -o pipefail
bash tools/gpucmd_r03t.sh || exit $?
bash tools/gpucmd_r03s.sh || exit $?
