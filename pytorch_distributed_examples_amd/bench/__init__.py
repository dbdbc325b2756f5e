"""Benchmark harness: :mod:`.harness` implements the root ``bench.py`` contract --
images/sec for the whole node on every BASELINE workload, N-rank launch and verification, hipGraph-recorded
steps, MAX-over-ranks timing, and the secondary ResNet-50 pipeline measurement at N >= 2."""
