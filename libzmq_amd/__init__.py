"""libzmq_amd: MI355X-native CurveZMQ MESSAGE AEAD path.

The product is libzmq_amd/libzmqg_curve.so (HIP kernels for gfx950 behind the
C ABI in include/zmqg_curve.h).  ``libzmq_amd.curve`` is its Python view.
"""
import os

PACKAGE_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PACKAGE_DIR, "libzmqg_curve.so")
