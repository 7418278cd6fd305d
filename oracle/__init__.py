"""CPU oracle of the vrpms hot path -- TEST INFRASTRUCTURE ONLY.

Imported only by ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py``.  ``spec.py`` is the pure-Python /
numpy restatement of the frozen semantic spec;
``oracle_c.c`` (built to ``liboracle.so`` by the Makefile) is its C
restatement used for large parity batches and the CPU baseline timing.
"""
