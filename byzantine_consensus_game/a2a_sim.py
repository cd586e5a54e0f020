"""Reference-layout shim: `import a2a_sim` from inside byzantine_consensus_game/."""
import _pkgpath  # noqa: F401
from byzantine_consensus_llm_agents_amd.bcg.a2a_sim import *  # noqa: F401,F403
