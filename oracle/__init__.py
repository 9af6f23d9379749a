"""CPU oracle for the rl4co-slap hot path -- TEST INFRASTRUCTURE ONLY.

This package is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import it.  The shipped package (``rl4co_slap_amd``) never imports it and fails
loudly when its HIP library is missing.

What it is
----------
A plain-PyTorch (CPU, float32/int64/bool/uint8 -- the reference dtypes)
restatement of the reference's hot path, written from the cited source lines of
``j4n1k/rl4co-slap`` (reference @ 2025-02-02):

* ``envs.py``      TSP / CVRP / SLAP ``_reset``/``_step``/``get_action_mask``/
                   ``get_reward``/``check_solution_validity`` and generators
                   (``rl4co/envs/routing/tsp/env.py:67-173``,
                   ``rl4co/envs/routing/cvrp/env.py:73-190``,
                   ``rl4co/envs/warehousing/slap/env.py:38-143``,
                   generators ``tsp/generator.py:51-60``,
                   ``cvrp/generator.py:116-143``, ``slap/generator.py:51-155``).
* ``ops.py``       ``rl4co/utils/ops.py:11-183`` (gather_by_index, tour length,
                   batchify/unbatchify, multistart helpers).
* ``decoding.py``  ``rl4co/utils/decoding.py:39-65,141-191,265-499``.
* ``rollout.py``   the decode loop ``rl4co/models/common/constructive/base.py:196-276``,
                   ``rollout`` (``decoding.py:88-109``), POMO shared baseline and
                   REINFORCE loss (``baselines.py:57-61``, ``reinforce.py:73-115``,
                   ``zoo/pomo/model.py:87-144``).
* ``td.py``        a dict-backed TensorDict stand-in (tensordict/torchrl are not
                   installed here) reproducing TorchRL's reset-merge semantics.

The SLAP per-batch Python loop (``slap/env.py:61-62``), the SLAP per-order loop
(``slap/env.py:136-142``), the CVRP per-step validity loop
(``cvrp/env.py:182-190``) and the double TSP validity sort
(``envs/common/base.py:186-187`` + ``tsp/env.py:158-159``) are kept on purpose:
this is also the CPU baseline that ``bench.py`` times.

Parity status
-------------
PARITY UNPINNED BY REFERENCE-HELD VECTORS.  The reference's own tests assert
shapes only (``tests/test_envs.py:56-59``, ``tests/test_policy.py:25-51``) and
hold no golden values; importing/running the reference in this pipeline was
denied.  The oracle is instead pinned by
(1) the reference's shape tests re-stated in ``tests/test_oracle.py``,
(2) hand-derived known-answer tests written from the cited source lines
    (``tests/test_oracle_kat.py``), and
(3) the reference's one value-level invariant test, the batchify round trip
    (``tests/test_utils.py:98-116`` of the reference).
Golden fixtures under ``tests/golden/`` are produced by this oracle
(``tests/golden/make_golden.py``) and are therefore self-consistent, not
reference-pinned.
"""
