"""Small test helpers mirroring kaolin/utils/testing.py:26-62."""
import functools
import random

import numpy as np
import torch

FLOAT_TYPES = [('cuda', torch.float), ('cuda', torch.double)]
FLOAT_DTYPES = [torch.float, torch.double]


def with_seed(torch_seed=0, numpy_seed=None, random_seed=None):
    def decorator(func):
        @functools.wraps(func)
        def wrapper(*args, **kwargs):
            torch.manual_seed(torch_seed)
            if numpy_seed is not None:
                np.random.seed(numpy_seed)
            if random_seed is not None:
                random.seed(random_seed)
            return func(*args, **kwargs)
        return wrapper
    return decorator
