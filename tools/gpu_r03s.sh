#!/bin/bash
# r03s: find_and_decode kernel timeline after the blind-decoder changes
set -e
export TMPDIR=/tmp
bash tools/trace_uedl.sh r03s
echo rc=0
