"""pyratslam_amd -- the pyratslam hot path (pose-cell network step and
view-template matcher) as hand-written HIP kernels for AMD Instinct MI355X
(gfx950), behind a C ABI (``include/ratslam_abi.h``) and drop-in Python classes
with the reference's API (``/root/reference/ratslam/posecell_network.py``,
``view_templates.py``).

    from pyratslam_amd import PoseCellNetwork, ViewTemplates
"""
from .posecell_network import PoseCellNetwork  # noqa: F401
from .view_templates import ShardedViewTemplates, ViewTemplate, ViewTemplates  # noqa: F401

__version__ = '0.1.0'
