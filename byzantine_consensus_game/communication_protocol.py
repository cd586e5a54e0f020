"""Reference-layout shim: `import communication_protocol` from inside byzantine_consensus_game/."""
import _pkgpath  # noqa: F401
from byzantine_consensus_llm_agents_amd.bcg.communication_protocol import *  # noqa: F401,F403
