"""Builds the host-side helper extension in-tree: fedml_amd/_host*.so (CPU code only).

The HIP kernels are NOT built here: they live in libfedagg.so (fedml_amd/csrc/Makefile, hipcc
--offload-arch=gfx950), a plain C-ABI library.  __graft_entry__.build() runs both.
"""
from setuptools import setup
from torch.utils.cpp_extension import BuildExtension, CppExtension

setup(
    name="fedml_amd",
    version="0.1.0",
    packages=["fedml_amd"],
    ext_modules=[CppExtension("fedml_amd._host", ["fedml_amd/csrc/host_tables.cpp"],
                              extra_compile_args=["-O3", "-std=c++17",
                                                  # host_sum.h: IEEE per-op rounding, never FMA
                                                  "-ffp-contract=off", "-fno-fast-math"])],
    cmdclass={"build_ext": BuildExtension},
)
