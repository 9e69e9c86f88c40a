"""ORACLE — test infrastructure only.

A CPU, float64 restatement of the reference's hot path (MoZhou1995/DeepPDE_ActorCritic:
equation.py and solver.py), written line by line against the reference and
citing the lines it follows.  It is the checker for the HIP path:

  * only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import it;
  * the product package ``deeppde_actorcritic_amd`` never imports it and has no
    CPU fallback.

Pinning status:
  * the samplers (equation.py:13-44) are pinned bit-for-bit against the
    reference's own sample_* methods, executed here with their real numpy/scipy
    dependencies (tests/golden/make_golden.py -> tests/golden/sampler_*.npz);
  * the analytic solutions are pinned by closed-form known-answer tests;
  * the rollout / TD / training-loop restatement is checked by invariants the
    reference code implies.  TensorFlow is not installed, so the TF-op level
    (rounding order inside tf.reduce_sum etc.) is **parity unpinned**.
"""
