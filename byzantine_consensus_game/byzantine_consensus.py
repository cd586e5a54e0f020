"""Reference-layout shim: `import byzantine_consensus` from inside byzantine_consensus_game/."""
import _pkgpath  # noqa: F401
from byzantine_consensus_llm_agents_amd.bcg.byzantine_consensus import *  # noqa: F401,F403
