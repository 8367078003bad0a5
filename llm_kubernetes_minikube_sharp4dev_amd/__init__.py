"""MI355X-native RAG / agent serving stack.

Capabilities of the ``Minimal_Agent`` / ``Minimal_RAG`` .NET demo
(reference: ``Minimal_Agent_RAG/*/Program.cs``) re-designed for AMD Instinct
MI355X (gfx950):

* ``rag``      – chunker / sanitizer / cosine index with the reference semantics,
                 GPU brute-force kNN (HIP) and a sharded multi-GPU index.
* ``agent``    – prompts, JSON extraction, tool dispatch and RAG gating.
* ``k8s``      – kubeconfig REST client for the 7 Kubernetes calls plus an
                 in-memory fake apiserver used by tests and benchmarks.
* ``apps``     – FastAPI ports of ``/health``, ``/rag/search``, ``/agent_rag`` and
                 ``/agent`` with identical JSON contracts.
* ``serving``  – an Ollama-compatible HTTP server (``/api/generate``,
                 ``/api/embeddings`` ...) so the unchanged C# solution can drive it.
* ``engine``   – paged-KV continuous-batching LLM engine with hipGraph decode,
                 embedding engine, samplers, constrained JSON decoding.
* ``models``   – Llama-3 / OPT decoders and BERT / bge / MiniLM / nomic-bert
                 encoders on top of ``ops``.
* ``ops``      – Python entry points of the hand-written CDNA4 HIP kernels
                 (``csrc/``), with fp32 torch references for CPU runs and tests.
* ``parallel`` – tensor parallelism over RCCL (torch.distributed ``nccl``),
                 data-parallel replica routing, sharded kNN.
* ``native``   – C++ runtime pieces (block allocator / scheduler core).
"""

__version__ = "0.1.0"

from . import config  # noqa: F401
