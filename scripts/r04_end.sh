#!/bin/bash
# round-4 end: the GPU suite + smoke, then the evidence (PMC, bench line, kernel trace, workloads)
set -o pipefail
bash scripts/r04_suite.sh && bash scripts/r04_final3.sh
