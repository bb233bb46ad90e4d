"""oracle/ -- CPU restatement of the reference's hot-path algorithms.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
`cpu_baseline` leg may import anything from here, and only as the checker (or the timed
CPU baseline) -- never as a product path.  The product (onetrainer_amd/) has no CPU
fallback and fails loudly without its HIP library.

Pinning (see DESIGN.md "Oracle"):
  * diffusion.py, adamw.py, lr.py -- pinned bit-for-bit (or to fp32 ulps where the
    reference's own float order is unobservable) against tests/golden/reference_math.npz,
    which tests/golden/make_golden.py produced by running the reference's own modules.
  * unet.py (diffusers UNet2DConditionModel restated) -- diffusers @5873377 is not in the
    image and no reference test pins the network: PARITY UNPINNED beyond the parameter-count
    and module-graph checks; train_step.py glue is pinned via fixtures.
"""
