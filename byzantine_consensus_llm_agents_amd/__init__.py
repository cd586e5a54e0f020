"""MI355X-native Byzantine Consensus Game framework.

Layers (see SURVEY.md §1 for the reference's layer map):
  bcg/       simulation layer, API-compatible with the reference
  engine/    in-process inference engine (scheduler, paged KV, JSON FSM, sampler)
  models/    Qwen3 / Qwen2 / Mistral decoders (TP-aware), weight loaders
  ops/       HIP/CDNA4 kernel bindings (+ PyTorch reference implementations)
  parallel/  RCCL tensor parallel + data-parallel launcher over seeds
  runtime/   native C++ runtime bindings (block manager, FSM compiler)
  utils/     timers, tracing, seeding
"""

__version__ = "0.1.0"
