"""Reference-layout shim: `import byzantine_consensus` from inside byzantine_consensus_game/."""
try:
    import _pkgpath  # noqa: F401  (run from inside byzantine_consensus_game/, as the reference)
except ImportError:  # imported as the package byzantine_consensus_game
    from . import _pkgpath  # noqa: F401
from byzantine_consensus_llm_agents_amd.bcg.byzantine_consensus import *  # noqa: F401,F403
