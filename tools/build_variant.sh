#!/bin/bash
# Build libiadmm.so from an alternative copy of the sources (variant studies; load it with
# IADMM_LIB_PATH=<out.so>).  Usage: [EXTRA="-DNAME=VAL ..."] bash tools/build_variant.sh <dir with csrc/> <out.so>
set -euo pipefail
src=$1; out=$2
obj=$(mktemp -d /tmp/var_obj_XXXX)
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -munsafe-fp-atomics -Wno-unused-result -mllvm -disable-promote-alloca-to-lds ${EXTRA:-}"
pids=()
for f in kkt lstm lstm_f16x3 admm ruiz lu gemm train metric_bwd probe; do
  /opt/rocm/bin/hipcc $FLAGS -c "$src/csrc/$f.hip" -o "$obj/$f.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$obj"/*.o -o "$out"
rm -rf "$obj"
echo "built $out"
