#!/bin/bash
# Build library variants for A/B runs: tools/variants.sh name "-DFLAG=.." [name "-D.." ...]
# -> hkd-mpc_amd/libhsddp_amd_<name>.so (same sources and flags as the Makefile, plus the defines)
set -e
cd "$(dirname "$0")/../hkd-mpc_amd/csrc"
FLAGS=$(make -s -p -n 2>/dev/null | sed -n 's/^FLAGS := //p' | head -1)
SRCS=$(make -s -p -n 2>/dev/null | sed -n 's/^SRCS := //p' | head -1)
while [ $# -ge 2 ]; do
    /opt/rocm/bin/hipcc $FLAGS $2 -shared -o ../libhsddp_amd_$1.so $SRCS &
    shift 2
done
wait
