# builds tools/diag_rollout (three CO_DIAG_PHASE variants of rollout.hip, symbols renamed)
set -e
cd "$(dirname "$0")"
for ph in 1 2 3; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -c \
    -DCO_DIAG_PHASE=$ph -Dco_tsp_rollout=diag${ph}_co_tsp_rollout -Dco_slap_rollout=diag${ph}_co_slap_rollout \
    -Dco_internal_tsp_reward_stepmajor=diag${ph}_internal \
    -I ../include ../rl4co_slap_amd/csrc/rollout.hip -o /tmp/diag_roll_$ph.o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 diag_rollout.cpp -x none /tmp/diag_roll_1.o /tmp/diag_roll_2.o /tmp/diag_roll_3.o -o diag_rollout
