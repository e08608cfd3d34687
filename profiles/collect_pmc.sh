#!/bin/bash
# PMC passes for the two dominant kernels (run through gpurun from the repo root):
#   bash profiles/collect_pmc.sh <tag>
# One rocprofv3 --pmc run per counter group (gfx950 slot limits: 8 SQ, 4 TCC
# with FETCH_SIZE = 3 and WRITE_SIZE = 2, 1 GRBM here). Workloads:
#   C4 (bench.py, C4 leg only)  -> pack_kernel<16>
#   C5 (tools/c5run.py C5: cold + warm run) -> lv_persist / lv_round / lv_insert
# Summaries: python3 profiles/pmc_sq.py gpurun_out/<tag> > profiles/<round>/pmc_sq.json
# (C5 under rocprofv3: the shipping cooperative launches, with tools/exit_hook.so (S2LC_EXIT_HOOK=1): the
# HIP runtime's own destructor faults at exit after cooperative launches under the profiler)
set -euo pipefail
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SHORT="--no-cpu-baseline --no-c5 --no-small --no-e2e --steps 3 --warmup 1"
pmc() {  # name, workload, counters...
  local name=$1 wl=$2; shift 2
  if [ "$wl" = c4 ]; then
    timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 bench.py $SHORT > "$OUT/$name.out" 2> "$OUT/$name.err"
  else
    S2LC_EXIT_HOOK=1 timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 tools/c5run.py C5 > "$OUT/$name.out" 2> "$OUT/$name.err"
  fi
}
pmc c4_sq_a c4 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE
pmc c4_sq_b c4 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES
pmc c5_sq_a c5 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE
pmc c5_fetch c5 FETCH_SIZE TCC_ATOMIC
pmc c5_write c5 WRITE_SIZE TCC_ATOMIC
pmc c5_atomic c5 TCC_ATOMIC TCC_EA0_ATOMIC
