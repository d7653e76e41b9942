#!/bin/bash
# Round 5: config 4's streamed apply, pipeline shapes (apply_pipe 0-3), arms alternated in one process.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 400 python -u tools/ab_kernel.py 4 bin_apply 3 - apply_pipe=0 apply_pipe=1 apply_pipe=3 > $O/ab_c4_pipe.txt 2>&1 || { tail -20 $O/ab_c4_pipe.txt; exit 1; }
cat $O/ab_c4_pipe.txt
