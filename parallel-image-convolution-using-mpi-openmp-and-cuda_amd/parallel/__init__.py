"""Multi-GPU row-band decomposition: bootstrap, RCCL halo engine, CPU emulator."""
