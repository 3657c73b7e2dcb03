"""CPU oracle (TEST INFRASTRUCTURE ONLY): clean-room NumPy restatement of the
reference's NLS readout, pinned to tests/golden/. Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg — never by deepfmkit_amd."""
