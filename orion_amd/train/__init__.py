"""Training engine: flat parameter arena, fused AdamW, data and checkpoints."""
