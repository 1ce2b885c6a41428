"""Drop-in for utils/random_tools.py: seed python, numpy and torch (default 35)."""
import random

import numpy as np
import torch


def fix_random(random_seed: int = 35) -> None:
    random.seed(random_seed)
    np.random.seed(random_seed)
    torch.manual_seed(random_seed)
    torch.cuda.manual_seed_all(random_seed)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
