"""drtc_amd: an MI355X-native distributed real-time chat & collaboration stack.

Layers (see SURVEY.md §1 for the reference's layer map):

* control plane (CPU): ``protos`` (wire contract), ``raft`` (consensus core,
  replicated chat state machine, persistence), ``server`` (gRPC services),
  ``client`` (CLI), ``llm`` (LLM service: prompts, parsers, engine backend);
* data plane (GPU): ``ops`` (HIP/CDNA4 kernels + torch references),
  ``models`` (Llama-3 / Gemma / Mixtral), ``engine`` (paged KV cache,
  continuous-batching scheduler, hipGraph decode), ``parallel`` (RCCL TP/EP,
  DP replica routing).
"""
__version__ = "0.1.0"
