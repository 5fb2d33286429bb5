"""Hot path: kernels/MMD^2 (mmd), scaling regulariser (ops), spectral norm (sn)."""
