"""oracle/ -- TEST INFRASTRUCTURE ONLY: the CPU restatement of OpenCV 3.4.1's CUDA TV-L1
(tvl1_oracle.c) and of its CPU DualTVL1 schedule (tvl1_oracle_dualtvl1.c).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this package, as the
checker -- never as the thing measured or shipped.  The product (fibsem-optflow_amd/) has
no path to it."""
