"""CPU oracle for the Sequential-VAE training step — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything from this package, and only as the checker / CPU
baseline.  The product path (``sequential-variational-autoencoder_amd``) never
imports, links or executes it.

What it restates
----------------
The executed training subgraph of ``sess.run([train_op, loss, final_loss])``
(``sequential_vae.py:1365``) of MWPainter/Sequential-Variational-Autoencoder:

* ``abstract_network.py:8-71``  — lrelu, conv2d_bn_lrelu, conv2d_t_bn(_relu),
  fc_bn_lrelu (TF-SAME conv / conv-transpose, training-mode BatchNorm with
  ``center=True, scale=False, eps=1e-3``).
* ``sequential_vae.py:877-1027`` — chain unroll, recognition + reparam sample.
* ``sequential_vae.py:1033-1093`` — generator wiring (training branch only).
* ``sequential_vae.py:1101-1212`` — per-step 16*MSE + reg*KL loss.
* ``sequential_vae.py:1537-1842`` — inference_ladder, generator_ladder,
  compute_encodings, split_latent, combine_noise('concat').
* ``sequential_vae.py:1246-1276`` + TF ``AdamOptimizer`` — clip + Adam.

Two independent restatements live here:

* ``model.py``  — numpy float64 forward with a tiny reverse-mode tape
  (``tape.py``) whose per-op backward formulas are written out by hand.
* ``torch_twin.py`` — the same graph in PyTorch-CPU autograd (fp32 or fp64);
  it is the cross-check of ``model.py`` and the CPU throughput baseline
  (``cpu_baseline.kind = "port"``).

Parity status: **parity unpinned**.  The reference needs TensorFlow 1.x with
``tf.contrib`` which is not installed (``import tensorflow`` ->
ModuleNotFoundError) and the reference ships no tests, fixtures
or golden vectors.  The oracle is therefore pinned only by (a) hand-computed
known-answer tests of the TF op semantics (tests/test_oracle_semantics.py),
(b) agreement of the two independent restatements, and (c) finite-difference
gradient checks.
"""
