"""CPU oracle (TEST INFRASTRUCTURE ONLY).

Restatement of the reference DiffusionDrive inference forward used to check the HIP path.
May be imported only by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg. The product package never imports it.
"""
