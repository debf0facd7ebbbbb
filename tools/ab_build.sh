#!/bin/bash
# Build A/B variants of libgrace_hip with extra -D defines: tools/ab_build.sh NAME DEF1,DEF2 ...
# -> grace_amd/lib/libgrace_hip_NAME.so
set -e
cd "$(dirname "$0")/.."
name=$1; defs=$2
GRACE_BUILD_DEFS="$defs" python3 grace_amd/build.py --variant=$name
