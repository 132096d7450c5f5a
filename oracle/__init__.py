"""CPU ORACLE -- test infrastructure only.

``oracle/`` restates the OpenCV 4.6 primitives (C, ``libvo_oracle.so``) and the
reference's orchestration (``vo_pipeline_oracle.py``) so that the HIP product can be
checked against them.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg import this package; the product package never does.
"""
