"""CPU oracle for the pyratslam hot path -- TEST INFRASTRUCTURE ONLY.

Nothing in ``pyratslam_amd`` imports this package.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import, call or link it, and only as the *checker* (or the timed CPU
baseline), never as the product path.

Contents
--------
``posecell``        NumPy restatement (float64) of ``PoseCellNetwork.update`` and
                    its helpers (``/root/reference/ratslam/posecell_network.py``)
                    plus the three OpenCL kernels it launches
                    (``/root/reference/ratslam/convolution.py:228-246,320-340,344-359``),
                    with the reference's accumulation order so results are
                    bit-identical to the reference's kernels compiled as host C.
``view_templates``  NumPy restatement of ``ViewTemplate.match`` / ``ViewTemplates``
                    (``/root/reference/ratslam/view_templates.py``), Python-2
                    integer-division semantics.
``c/``              C restatement (float64 / uint64, OpenMP) of the same kernels;
                    built into ``oracle/lib/libratslam_oracle.so`` and used as the
                    multi-core CPU baseline.

Pinning
-------
The restatement is pinned against outputs of the reference itself, run in the
build container: ``tests/golden/gen_golden.py`` imports the reference modules
(with Py2 shims), JIT-compiles the reference's own OpenCL kernel text as host C
and records kernels, LUTs, pose-cell trajectories and template-match traces as
``tests/golden/*.npz``.  ``tests/test_oracle_golden.py`` checks the oracle
against every one of those vectors (bit-exact).
"""
