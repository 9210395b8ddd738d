"""ORACLE — test infrastructure only.

CPU restatements of the reference's hot path used as the parity checker (tests/,
__graft_entry__.smoke(), bench.py's cpu_baseline leg).  The product (libzasr.so and the
sherpa-vietnamese-asr_amd/ host package) never imports, links or executes anything here.
"""
