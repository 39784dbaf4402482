"""kgs.serve -- Llama serving on the kgs kernels (BASELINE config 5 stand-in for
``pods/vllm-rocm-pod.yaml``: Llama-3-8B bf16, TP=1, one MI355X).

* :class:`LLMEngine` (engine.py): native continuous-batching scheduler
  (``native/serve/scheduler.cpp``), paged KV cache, hipGraph decode steps;
* :class:`ServingModel` (model.py): prefill on the 256x256 MFMA GEMM + flash
  attention, decode on the skinny GEMM + paged decode attention;
* ``python -m kgs.serve serve`` (api.py): OpenAI-style HTTP server;
* ``python -m kgs.serve bench`` (bench.py): offline throughput benchmark.
"""
from .engine import EngineConfig, LLMEngine, Request, SamplingParams  # noqa: F401
from .model import ServingModel  # noqa: F401
