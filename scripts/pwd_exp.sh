#!/bin/bash
# Build timing-experiment variants of libdorknet_hip.so with pw_deep.hip compiled under
# -DDK_PWD_EXP=<bits> (see pw_deep.hip), into dorknet_amd/lib/exp<bits>/ (run with
# DORKNET_HIP_LIB=...).  Usage: bash scripts/pwd_exp.sh 1 2 8
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$ROOT/dorknet_amd/lib/obj
for b in "$@"; do
  D=$ROOT/dorknet_amd/lib/exp$b; mkdir -p "$D"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -DDK_PWD_EXP=$b \
      -c "$ROOT/dorknet_amd/csrc/pw_deep.hip" -o "$D/pw_deep.o"
  OBJS=$(ls "$OBJ"/*.o | grep -v '/pw_deep.o$')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o "$D/libdorknet_hip.so" $OBJS "$D/pw_deep.o"
  rm -f "$D/pw_deep.o"
  echo "built $D"
done
