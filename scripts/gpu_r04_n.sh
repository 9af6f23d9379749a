# Round 4 pass n: the fused CVRP decode + env step alone, new (branch-free row loads,
# unconditional staged reads) against the previous decode_env object, interleaved.
cd $GRAFT_REPO_ROOT
for p in 1 2 3; do
  timeout -k 10 120 python3 tools/diag_cvrp_fused.py || exit 1
  CO_LIB=tools/_variants/libco_env_oldenv.so timeout -k 10 120 python3 tools/diag_cvrp_fused.py | sed 's/^/old: /' || exit 1
done
