#!/bin/bash
# Diagnostic builds of the library with alternative tuning macros (not the product):
#   tools/build_variants.sh NAME "-DFOO=1 -DBAR=2" ...  -> tools/_variants/libco_env_NAME.so
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_variants
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
    -fno-fast-math -Iinclude $2 -o tools/_variants/libco_env_$1.so \
    rl4co_slap_amd/csrc/{tsp,cvrp,slap,ops,decode,rollout,nearest}.hip &
  shift 2
done
wait
