"""Oracle package: CPU restatement of the reference (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  See ca_lanczos_ref.py for the parity status.
"""
