"""Reference-layout entry point: ``python main.py --honest 8 --byzantine 2``.

Same CLI as the reference ``byzantine_consensus_game/main.py``; the work is done
by :mod:`byzantine_consensus_llm_agents_amd.bcg.main`.
"""
try:
    import _pkgpath  # noqa: F401  (run from inside byzantine_consensus_game/, as the reference)
except ImportError:  # imported as the package byzantine_consensus_game
    from . import _pkgpath  # noqa: F401
from byzantine_consensus_llm_agents_amd.bcg.main import main, run_simulation  # noqa: F401
from byzantine_consensus_llm_agents_amd.bcg.simulation import BCGSimulation, tee_print  # noqa: F401

if __name__ == "__main__":
    main()
