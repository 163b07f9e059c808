"""ORACLE — test infrastructure only.

CPU restatement of GNSS-SDR's acquisition (pcps_acquisition) and tracking
multicorrelator (VOLK-GNSSSDR generic protokernels) used as the parity checker by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing in the
product package (gnss-sdr-new_amd/) imports, links or executes anything here.
"""
