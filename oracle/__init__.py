"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's numerical renderer.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package,
and only as the checker / the timed CPU baseline.  The product path (nlos-gaussian-renderer_amd/)
never imports it and fails loudly when its HIP library is missing.

Parity pinning: oracle/torch_ref.py is checked against golden vectors produced by running the
reference's own PyTorch path (tests/golden/make_golden.py, imported from /root/reference in the
build container) — see tests/test_oracle_golden.py.  The "cuda" preset (semantics of
submodules/cuda_renderer/src/volume_renderer.cu) and the analytic section path cannot run in
the reference here (no NVIDIA toolchain), so those restatements are *parity unpinned* beyond
their line-by-line citation of the .cu sources.
"""
