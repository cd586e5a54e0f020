"""Reference-layout shim: `import protocol_factory` from inside byzantine_consensus_game/."""
import _pkgpath  # noqa: F401
from byzantine_consensus_llm_agents_amd.bcg.protocol_factory import *  # noqa: F401,F403
