"""Build the native extension ``upow_amd/_native*.so`` in-tree for gfx950.

* ``csrc/*.hip`` -> ``hipcc --offload-arch=gfx950 -O3`` (device + host code)
* ``csrc/*.cpp`` -> host C++ (pybind11 bindings, CPU crypto)
* link with ``hipcc -shared`` (libamdhip64)

Objects are cached by content hash of the source + all headers, so re-running is cheap.
Usage: ``python -m upow_amd._build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / 'csrc'
BUILD = ROOT / 'build' / 'native'
PKG = ROOT / 'upow_amd'
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
# host-only C++: ROCm's clang++, the compiler hipcc drives for the device files (one toolchain; its code for
# the codec's base58 and SHA paths is 10-30 % faster than g++ -O3 here)
CXX = os.environ.get('CXX', '/opt/rocm/llvm/bin/clang++')
ARCH = os.environ.get('UPOW_OFFLOAD_ARCH', 'gfx950')
EXT_SUFFIX = sysconfig.get_config_var('EXT_SUFFIX') or '.so'
TARGET = PKG / f'_native{EXT_SUFFIX}'


def _pybind_include() -> str:
    import pybind11
    return pybind11.get_include()


def _headers_digest() -> str:
    h = hashlib.sha256()
    for p in sorted(CSRC.glob('*.h')):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def _flags_common():
    return ['-O3', '-std=c++17', '-fPIC', '-Wall', '-Wno-unused-function', f'-I{CSRC}']


# Sanitizer variants (tools/sanitize_host.sh): the same sources, host code instrumented, linked into
# build/native-<variant>/_native*.so and loaded by an instrumented embedded interpreter (tools/pysan.c)
# through UPOW_NATIVE_SO. Device code keeps -O3; the HIP TUs' host side is instrumented at -O0 (the
# force-inlined 256-bit field code takes ~10 min to optimise under instrumentation).
SAN_FLAGS = {'asan': ['-fsanitize=address,undefined', '-fno-sanitize-recover=undefined'],
             'tsan': ['-fsanitize=thread']}
CLANGXX = '/opt/rocm/llvm/bin/clang++'


# Per-file device code generation. The P-256 kernels are long chains of dependent 64-bit multiply-adds and
# carry chains; gfx950 needs wait states between a v_mad_u64_u32 and the first read of its result, which the
# default (occupancy-first) scheduler fills with s_nop: 6,865 of the quad verify kernel's 42,629 static
# instructions. The ILP-first machine scheduler interleaves independent products instead (1,810 s_nop): the
# block-latency kernels run one wave per SIMD, so the extra registers cost them nothing; the batch kernels
# keep their __launch_bounds__ occupancy.
DEVICE_FLAGS = {'p256': ['-mllvm', '-amdgpu-sched-strategy=max-ilp']}  # p256_batch.hip: the default schedule
# A/B builds of the P-256 kernels (build-ab/native-<variant>, shipped to the GPU box and loaded through
# UPOW_NATIVE_SO): 'p256occ' the occupancy-first schedule, 'p256bgcd' the binary-Euclid s^-1,
# 'p256batchilp' the one-lane batch kernel under the ILP-first schedule too
AB_VARIANTS = {'p256occ': {'p256': []}, 'p256bgcd': {'p256': DEVICE_FLAGS['p256'] + ['-DUPOW_P256_INV_BGCD=1']},
               'p256batchilp': {'p256_batch': ['-mllvm', '-amdgpu-sched-strategy=max-ilp']}}


def _device_flags(src: Path, variant: str) -> list:
    if variant in AB_VARIANTS:
        return AB_VARIANTS[variant].get(src.stem, DEVICE_FLAGS.get(src.stem, []))
    return DEVICE_FLAGS.get(src.stem, [])


def _build_dir(variant: str) -> Path:
    if variant in AB_VARIANTS:  # shipped to the GPU box for the A/B (./build is not)
        return ROOT / 'build-ab' / f'native-{variant}'
    return BUILD if variant == 'release' else ROOT / 'build' / f'native-{variant}'


def _compile(src: Path, hdr_digest: str, force: bool, variant: str = 'release') -> Path:
    out = _build_dir(variant)
    out.mkdir(parents=True, exist_ok=True)
    dev = _device_flags(src, variant) if src.suffix == '.hip' else []
    key = hashlib.sha256(src.read_bytes() + hdr_digest.encode() + ARCH.encode() + variant.encode()
                         + ' '.join(dev).encode() + (CXX.encode() if src.suffix != '.hip' else b'')).hexdigest()[:16]
    obj = out / f'{src.stem}.{key}.o'
    if obj.exists() and not force:
        return obj
    san = SAN_FLAGS.get(variant)
    if src.suffix == '.hip':
        host = [] if san is None else ['-Xarch_host', '-O0', '-Xarch_host', '-g1',
                                       *[x for f in san for x in ('-Xarch_host', f)]]
        cmd = [HIPCC, f'--offload-arch={ARCH}', *_flags_common(), *dev, *host, '-c', str(src), '-o', str(obj)]
    else:
        # host-only translation units: plain C++ (no device pass)
        cxx, extra = (CXX, []) if san is None else (CLANGXX, ['-O1', '-g', '-fno-omit-frame-pointer', *san])
        cmd = [cxx, *_flags_common(), *extra, f'-I{_pybind_include()}', f'-I{sysconfig.get_paths()["include"]}',
               '-I/opt/rocm/include', '-fvisibility=hidden', '-c', str(src), '-o', str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'compile failed: {" ".join(cmd)}\n{r.stdout}\n{r.stderr}')
    return obj


def build(force: bool = False, jobs: int = 4, verbose: bool = True, variant: str = 'release') -> Path:
    """Compile and link the extension; ``variant`` 'asan' / 'tsan' builds an instrumented copy under
    build/native-<variant>/ (the in-tree release .so is untouched)."""
    srcs = sorted(CSRC.glob('*.hip')) + sorted(CSRC.glob('*.cpp'))
    hd = _headers_digest()
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, hd, force, variant), srcs))
    target = TARGET if variant == 'release' else _build_dir(variant) / TARGET.name
    link_key = hashlib.sha256(''.join(o.name for o in objs).encode()).hexdigest()[:16]
    stamp = _build_dir(variant) / 'link.stamp'
    if target.exists() and stamp.exists() and stamp.read_text() == link_key and not force:
        if verbose:
            print(f'[upow_amd._build] up to date: {target.name}')
        return target
    TARGET_ = target
    # instrumented variants leave the sanitizer runtime to the executable that loads them (tools/pysan.c)
    cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', str(TARGET_), *map(str, objs), '-ldl']
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'link failed: {" ".join(cmd)}\n{r.stdout}\n{r.stderr}')
    stamp.write_text(link_key)
    if verbose:
        print(f'[upow_amd._build] built {TARGET_} from {len(objs)} objects')
    return TARGET_


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--force', action='store_true')
    ap.add_argument('-j', '--jobs', type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument('--variant', choices=['release', 'asan', 'tsan', *AB_VARIANTS], default='release')
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs, variant=a.variant)


if __name__ == '__main__':
    sys.exit(main())
