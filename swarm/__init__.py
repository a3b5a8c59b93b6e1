"""CLI-compatible entry points of the reference worker (``python -m swarm.worker``,
``python -m swarm.initialize``, ``python -m swarm.test``; reference:
.vscode/launch.json:14-37, Dockerfile:37).  The implementation lives in
``chiaswarm_amd``."""
from chiaswarm_amd import __version__  # noqa: F401
