#!/bin/bash
# round-6 evidence (from the repo root via gpurun): bench, rocprofv3 kernel
# stats of C4 and C5, C4 HBM PMC, the SQ / FETCH / WRITE / atomic PMC passes
# of both workloads, and their summaries
set -euo pipefail
TAG=${1:-r06p}
bash profiles/collect.sh "$TAG"
bash profiles/collect_pmc.sh "$TAG/pmc"
python3 profiles/pmc_c5.py "gpurun_out/$TAG/pmc" > "gpurun_out/$TAG/pmc_c5.json"
python3 profiles/pmc_sq.py "gpurun_out/$TAG/pmc" > "gpurun_out/$TAG/pmc_sq.json"
