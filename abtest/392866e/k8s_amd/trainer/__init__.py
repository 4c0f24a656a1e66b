"""TfJob workload runtime (``python -m k8s_amd.trainer``); see ``runner.py``."""
from k8s_amd.trainer.runner import main  # noqa: F401
