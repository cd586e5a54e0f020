"""Byzantine Consensus Game simulation layer (API-compatible with the reference).

Modules mirror the reference's flat layout (``config``, ``byzantine_consensus``,
``a2a_sim``, ``agent_network``, ``communication_protocol``, ``protocol_factory``,
``bcg_agents``, ``main``) plus ``engine_agent`` (the in-process MI355X engine
adapter that replaces ``vllm_agent``).
"""
