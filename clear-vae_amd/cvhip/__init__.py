"""cvhip — host side of libclearvae_hip.so (the MI355X CLEAR-VAE hot path).

_lib      ctypes binding of the C-ABI in include/clearvae.h (no CPU fallback)
plan      layer plan, flat parameter arena, device workspaces, call programs
autograd  torch.autograd.Function wrappers used by the reference-API modules in src/
engine    fused trainer step (HIP graph replay) used by src.trainer
dist      data-parallel plumbing (broadcast, bucketed gradient all-reduce)
rng       device RNG offsets and the test-only noise/permutation injection queues
"""
