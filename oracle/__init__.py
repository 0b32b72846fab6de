"""oracle/ -- TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's hot path (tridang04022004/UG-PG-UNet), used as
the parity checker for the HIP product path.  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
package.  The product package (`ug-pg-unet_amd/ugpg`) never imports it and has
no CPU fallback.

Parity status: PINNED.  `oracle/make_goldens.py` imports the reference from
/root/reference in the build container, checks `ref_cpu` against it with
`torch.equal` on identical inputs/weights, and writes the golden fixtures under
`tests/golden/` that the CPU test-suite re-checks on every run.
"""
