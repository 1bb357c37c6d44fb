"""lie_vae — MI355X-native drop-in for the SO(3) latent hot path of pimdh/lie-vae.

Modules: ``lie_tools`` (SO(3) maps, Wigner-D action), ``reparameterize`` (N0 / SO(3)
reparameterisers and mean modules), ``decoders`` (ActionNet), ``utils``.  The compute
runs in ``liblievae_hip.so`` (HIP, gfx950) through a C ABI (include/lievae.h).
"""
__version__ = "0.1.0"
