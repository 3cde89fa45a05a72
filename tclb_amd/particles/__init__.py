"""Particle coupling (reference: RemoteForceInterface + simplepart + SolidContainer,
src/RemoteForceInterface.*, src/simplepart.cpp, src/Particle.hpp).

MI355X-native design: the particle set lives in one process per GPU next to the
lattice; positions/velocities are uploaded to device memory before every particle
stage (a few KB), the stage kernel (model ``CalcF`` through ``ParticleLoop``)
accumulates force and moment per particle with wave-reduced atomics, the sums are
all-reduced across ranks (RCCL/gloo) and the built-in rigid-body integrator
("SimplePart") advances the particles.  No MPMD intercommunicator is needed.
An integrator that runs as another program (a DEM code, tools/rfi_simplepart.py)
couples through the socket RFI bridge in ``rfi.py``.
"""
from .system import ParticleSystem, SimplePart, integrate_rigid  # noqa: F401
from .rfi import IntegratorClient, RemoteParticles  # noqa: F401
