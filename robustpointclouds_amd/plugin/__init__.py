"""Drop-in plugin surface with the reference's import paths.

Put this directory on sys.path and the reference's configs resolve
unchanged: `custom_imports=['models', 'models.detectors.adversarial_voxelnet',
'models.adversarial.voxel_perturber', 'custom_hook']` import the modules below, which
register `AdversarialVoxelNet`, `AdversarialCenterPoint`, `VoxelPerturber` and the hooks
into mmengine/mmdet3d registries when those are installed, or into
robustpointclouds_amd.registry otherwise.
"""
import os

PLUGIN_DIR = os.path.dirname(os.path.abspath(__file__))
