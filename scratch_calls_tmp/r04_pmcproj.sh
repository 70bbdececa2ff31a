#!/bin/bash
# Round-4 tree: PMC passes (tools/calls/r03_pmc.sh) then the N = 8 slice projection (tools/projection_final.sh).
set -e -o pipefail
bash tools/calls/r03_pmc.sh ${1:-r04pmc}/pmc
bash tools/projection_final.sh ${1:-r04pmc}/proj
