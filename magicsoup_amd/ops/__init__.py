"""Native operator layer: HIP (gfx950) kernels and the OpenMP host core, plus device dispatch."""
