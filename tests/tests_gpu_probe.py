import os


def gpu_present():
    """True when /dev/kfd exists and torch sees a HIP device (without initialising HIP otherwise)."""
    if not os.path.exists("/dev/kfd"):
        return False
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False
