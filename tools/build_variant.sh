#!/bin/bash
# Build a diagnostic variant of libtsrl.so with extra -D flags for ONE source file:
#   tools/build_variant.sh <name> <source.hip> <flags...>   -> variants/libtsrl_<name>.so
# (load it with TSRL_LIB_PATH=variants/libtsrl_<name>.so)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; src=$2; shift 2
PKG=$ROOT/tianshou-fork_amd
make -C "$PKG" -s
mkdir -p "$ROOT/variants/obj_$name"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics"
objs=""
for o in "$PKG"/build/obj/*.o; do
  b=$(basename "$o" .o)
  if [ "$b" = "$(basename "$src")" ]; then
    /opt/rocm/bin/hipcc $FLAGS "$@" -c -o "$ROOT/variants/obj_$name/$b.o" "$PKG/csrc/$(basename "$src")"
    objs="$objs $ROOT/variants/obj_$name/$b.o"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/variants/libtsrl_$name.so" $objs
rm -rf "$ROOT/variants/obj_$name"
echo "built variants/libtsrl_$name.so"
