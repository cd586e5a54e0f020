"""Reference-layout shim: `import config` from inside byzantine_consensus_game/."""
import _pkgpath  # noqa: F401
from byzantine_consensus_llm_agents_amd.bcg.config import *  # noqa: F401,F403
