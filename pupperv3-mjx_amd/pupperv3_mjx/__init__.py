"""pupperv3_mjx (MI355X-native): the PupperV3 locomotion env hot path as HIP kernels.

Module names mirror the reference package (environment, config, domain_randomization,
obstacles, utils) so an upstream training script can switch by changing its import root.
"""
import os

ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")
MODEL_XML = os.path.join(ASSET_DIR, "pupper_v3.xml")
