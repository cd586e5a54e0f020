"""Reference-layout shim: `import bcg_agents` from inside byzantine_consensus_game/."""
try:
    import _pkgpath  # noqa: F401  (run from inside byzantine_consensus_game/, as the reference)
except ImportError:  # imported as the package byzantine_consensus_game
    from . import _pkgpath  # noqa: F401
from byzantine_consensus_llm_agents_amd.bcg.bcg_agents import *  # noqa: F401,F403
from byzantine_consensus_llm_agents_amd.bcg.bcg_agents import print, verbose_print, set_agent_log_file  # noqa: F401,E402
