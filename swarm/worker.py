"""``python -m swarm.worker`` — the worker daemon (chiaswarm_amd.runtime.worker)."""
from chiaswarm_amd.runtime.worker import main

if __name__ == "__main__":
    main()
