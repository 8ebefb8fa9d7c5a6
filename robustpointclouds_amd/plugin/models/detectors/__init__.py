from .adversarial_centerpoint import AdversarialCenterPoint  # noqa: F401
from .adversarial_voxelnet import AdversarialVoxelNet  # noqa: F401
from .strong_adversarial_voxelnet import StrongAdversarialVoxelNet  # noqa: F401

__all__ = ["AdversarialVoxelNet", "StrongAdversarialVoxelNet", "AdversarialCenterPoint"]
