"""orion_amd -- an MI355X-native rebuild of the Oríon asynchronous black-box
(hyper-parameter) optimization framework, with a GPT-2/Llama training workload
on hand-written gfx950 HIP kernels and RCCL data parallelism.

Subpackages
-----------
space      search-space dimensions and the ``~`` prior DSL
algo       optimization algorithms (random search, gradient descent, plugins)
store      document stores with compare-and-swap (memory, SQLite, MongoDB)
core       trials, experiments, producer/consumer, worker loop, CLI, config
client     ``report_results`` for user scripts
models     GPT-2 and Llama decoders
ops        fused HIP kernels (+ PyTorch reference implementations)
parallel   RCCL data-parallel reducer, launch helpers
train      flat-arena trainer, fused AdamW, data, checkpoints
utils      registry, logging, timers
"""
__version__ = "0.1.0"
__descr__ = "Distributed Asynchronous [black-box] Optimization on MI355X"
