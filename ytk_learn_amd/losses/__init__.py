from .functions import LossFunction, create_loss, pure_classification  # noqa: F401
