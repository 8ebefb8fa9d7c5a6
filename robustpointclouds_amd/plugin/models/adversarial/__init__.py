from .voxel_perturber import VoxelPerturber  # noqa: F401

__all__ = ["VoxelPerturber"]
