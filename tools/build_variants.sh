#!/bin/bash
# Diagnostic builds of the library with alternative tuning macros (not the product):
#   tools/build_variants.sh [-s cvrp] NAME "-DFOO=1 -DBAR=2" ...  -> tools/_variants/libco_env_NAME.so
# With -s SRC only SRC.hip is recompiled with the macros; the other objects come from
# the product build (rl4co_slap_amd/_lib/obj, run `python -m rl4co_slap_amd.csrc.build` first).
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_variants
ONLY=""
if [ "$1" = "-s" ]; then ONLY=$2; shift 2; fi
ALL="tsp cvrp slap ops decode_step decode_tsp decode_env rollout nearest"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Iinclude"
while [ $# -ge 2 ]; do
  if [ -n "$ONLY" ]; then
    (
      objs=""
      for s in $ALL; do
        if [ "$s" = "$ONLY" ]; then
          /opt/rocm/bin/hipcc $FLAGS $2 -c rl4co_slap_amd/csrc/$s.hip -o tools/_variants/$1_$s.o
          objs="$objs tools/_variants/$1_$s.o"
        else
          objs="$objs rl4co_slap_amd/_lib/obj/$s.o"
        fi
      done
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_variants/libco_env_$1.so -x none $objs
    ) &
  else
    /opt/rocm/bin/hipcc $FLAGS -shared $2 -o tools/_variants/libco_env_$1.so \
      rl4co_slap_amd/csrc/{tsp,cvrp,slap,ops,decode_step,decode_tsp,decode_env,rollout,nearest}.hip &
  fi
  shift 2
done
wait
