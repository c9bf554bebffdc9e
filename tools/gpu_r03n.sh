#!/bin/bash
# r03n: ue_dl host phase timing (run_frontend split) + timeline
set -e
export TMPDIR=/tmp
bash tools/trace_uedl.sh r03n
echo rc=0
