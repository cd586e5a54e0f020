"""Reference-layout shim: `import engine_agent` from inside byzantine_consensus_game/."""
try:
    import _pkgpath  # noqa: F401  (run from inside byzantine_consensus_game/, as the reference)
except ImportError:  # imported as the package byzantine_consensus_game
    from . import _pkgpath  # noqa: F401
from byzantine_consensus_llm_agents_amd.bcg.engine_agent import *  # noqa: F401,F403
