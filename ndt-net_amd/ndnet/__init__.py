"""ndnet (MI355X): the NDT preprocessing + NDTNet forward path of NDT-Net on gfx950.

Mirrors the reference package layout so that ``from ndnet.preprocessing...``
and ``from ndnet.models.ndtnet ...`` resolve here when ``ndt-net_amd/`` is on
``sys.path``.
"""
__version__ = "0.1.0"
