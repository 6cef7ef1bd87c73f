"""Multi-GPU execution: RCCL data parallelism over xGMI."""
