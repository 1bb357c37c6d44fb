"""Callers of the hot path: network blocks (nets), the VAE glue (vae) and the
data-parallel trainer (train_dp).  Convs stay on PyTorch-ROCm (MIOpen/hipBLASLt)."""
