#!/bin/bash
# Dev tool: build libzasr.so with one translation unit compiled under extra flags, into
# ablib/NAME/libzasr.so (A/B runs select it with ZASR_LIB).  Run after `make` in csrc/.
# usage: ab_variant.sh NAME SRC.hip "-DFLAG=..."
set -e
N=$1; SRC=$2; FL=$3
C=$(dirname $0)/../csrc; B=$C/../build; O=/tmp/abv_$N; mkdir -p $O $(dirname $0)/../../ablib/$N
extra=""; [ "$SRC" = attn_kernels.hip ] && extra="-mllvm -amdgpu-mfma-vgpr-form"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $extra $FL -c $C/$SRC -o $O/${SRC%.hip}.o
objs=""; for o in $B/*.o; do b=$(basename $o); [ "$b" = "${SRC%.hip}.o" ] && objs="$objs $O/$b" || objs="$objs $o"; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $(dirname $0)/../../ablib/$N/libzasr.so $objs
echo built ablib/$N
