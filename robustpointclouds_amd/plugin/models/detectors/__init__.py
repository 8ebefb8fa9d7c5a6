from .adversarial_voxelnet import AdversarialVoxelNet  # noqa: F401

__all__ = ["AdversarialVoxelNet"]
