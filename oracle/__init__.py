"""ORACLE — test infrastructure only.

CPU restatement (PyTorch CPU, fp32) of the reference's search-over-noise path,
used exclusively as the CHECKER by ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py``. The product path (the ``itsd`` package and
its HIP library) never imports anything from here.

Parity status: PINNED — ``tests/golden/*.npz`` hold outputs of the reference
itself (imported by file path from /root/reference in the build container by
``tools/gen_golden.py``), and ``tests/test_oracle_golden.py`` checks this
restatement against them.
"""
