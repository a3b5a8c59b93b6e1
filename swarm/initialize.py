"""``python -m swarm.initialize [--reset] [--silent]`` (chiaswarm_amd.initialize)."""
from chiaswarm_amd.initialize import main

if __name__ == "__main__":
    main()
