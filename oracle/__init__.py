"""CPU oracle for the U-Net hot path (test infrastructure only; see keras_ops.py header).

PARITY UNPINNED: the reference ships no golden data and its TensorFlow runtime is absent.
"""
