import sys

from k8s_amd.trainer.runner import main

if __name__ == "__main__":
    sys.exit(main())
