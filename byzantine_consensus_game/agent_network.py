"""Reference-layout shim: `import agent_network` from inside byzantine_consensus_game/."""
import _pkgpath  # noqa: F401
from byzantine_consensus_llm_agents_amd.bcg.agent_network import *  # noqa: F401,F403
