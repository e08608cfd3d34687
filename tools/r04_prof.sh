#!/bin/bash
# round-4 evidence: bench, kernel stats, C4 PMC, C5 stats, PMC passes + summaries
set -euo pipefail
TAG=${1:-r04p}
bash profiles/collect.sh "$TAG"
bash profiles/collect_pmc.sh "$TAG/pmc"
python3 profiles/pmc_c5.py "gpurun_out/$TAG/pmc" > "gpurun_out/$TAG/pmc_c5.json"
python3 profiles/pmc_sq.py "gpurun_out/$TAG/pmc" > "gpurun_out/$TAG/pmc_sq.json"
