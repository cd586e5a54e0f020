"""Reference-layout shim: `import engine_agent` from inside byzantine_consensus_game/."""
import _pkgpath  # noqa: F401
from byzantine_consensus_llm_agents_amd.bcg.engine_agent import *  # noqa: F401,F403
