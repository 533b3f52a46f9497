"""pnp_amd — MI355X-native batched kinematics / DLS-IK engine for the panda_mujoco_gym scene.

Host package over libpnp.so (HIP kernels for gfx950, C ABI in include/pnp.h).  Importing the
package does not touch the GPU; the library is loaded on first use and its absence is an error.
"""
from .model import PandaModel, load_model  # noqa: F401

__all__ = ["PandaModel", "load_model"]
