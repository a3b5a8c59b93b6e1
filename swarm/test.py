"""``python -m swarm.test [job]`` — manual smoke job (chiaswarm_amd.smoke)."""
from chiaswarm_amd.smoke import main

if __name__ == "__main__":
    main()
