from torch.optim.lr_scheduler import StepLR

from .adadelta import Adadelta

__all__ = ["Adadelta", "StepLR"]
