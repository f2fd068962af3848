"""Build libcurvezmq_mi355x.so in-tree for gfx950 with hipcc (no JIT cache, no torch extension).

The .so lands next to this file so it travels to the GPU box with the repo
snapshot and is what jeromq_amd._lib loads.

Every build is gated on the device ISA of the binary it produced (`isa_gate`): the gfx950 code
objects are cut out of the linked library's .hip_fatbin, disassembled with llvm-objdump, and
scanned by tools/isa_store_hazard.py for the VMEM store hazards the compiler does not count
(store data rewritten at distance 1, a VALU-written SGPR read by VMEM within 5 states, a wide
buffer store with a register soffset: DESIGN.md section 6).  A hit leaves the previous library in
place and raises: a hazard in the shipped kernels writes wrong bytes silently.
"""
import os
import shutil
import struct
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
PRODUCT_LIB = os.path.join(HERE, "libcurvezmq_mi355x.so")
LIB = os.environ.get("CZ_LIB_OUT", PRODUCT_LIB)
# "file#n": the file compiled with -DCZ_KPART=n (cz_kernels.hip builds as three parts in parallel)
SOURCES = ["cz_kernels.hip#1", "cz_kernels.hip#2", "cz_kernels.hip#3", "cz_x25519.hip", "cz_host.cpp", "cz_mechanism.cpp", "cz_wire.cpp", "cz_engine.cpp", "cz_handshake.cpp", "cz_curve_hs.cpp"]
HEADERS = ["cz_device.h", "cz_diag.h", "cz_internal.h", "cz_salsa_lazy.h", "cz_salsa_tail.h", os.path.join("..", "..", "include", "curvezmq_mi355x.h")]
ARCH = os.environ.get("CZ_OFFLOAD_ARCH", "gfx950")
LLVM_BIN = "/opt/rocm/lib/llvm/bin"
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


class IsaHazardError(RuntimeError):
    pass


class ProductFlagsError(ValueError):
    """Extra compile flags (A/B variants, wrong-output diagnostics) asked for the product library."""


def compile_flags(lib, extra_env=None):
    """hipcc flags for `lib`.  The product library (jeromq_amd/libcurvezmq_mi355x.so, what
    jeromq_amd._lib loads and the GPU box runs) is built with exactly the committed flags plus
    -DCZ_PRODUCT_BUILD: CZ_EXTRA_FLAGS is refused for it, so a variable left set on a build box can
    never ship an A/B variant or a wrong-output diagnostic (cz_diag.h also #errors on one).  A/B
    builds name another output with CZ_LIB_OUT (tools/build_variant.sh)."""
    raw = os.environ.get("CZ_EXTRA_FLAGS", "") if extra_env is None else extra_env
    extra = raw.split()
    product = os.path.realpath(lib) == os.path.realpath(PRODUCT_LIB)
    if product and extra:
        raise ProductFlagsError(f"CZ_EXTRA_FLAGS={raw!r} refused for the product library {PRODUCT_LIB}: "
                                "A/B builds set CZ_LIB_OUT to another path")
    common = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall"]
    return common + (["-DCZ_PRODUCT_BUILD"] if product else extra)


def _stale(lib=LIB, sources=SOURCES):
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(os.path.join(CSRC, f.split("#")[0])) > t for f in list(sources) + HEADERS)


def device_code_objects(so_path, arch=ARCH):
    """The `arch` code objects (ELF) inside a HIP library's .hip_fatbin: one offload bundle per
    translation unit, each `magic, u64 n, n x {u64 offset, u64 size, u64 triple_len, triple}`
    with offsets from the bundle's start."""
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run([os.path.join(LLVM_BIN, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fb}", so_path,
                        os.path.join(td, "discard")], check=True, capture_output=True)
        data = open(fb, "rb").read()
    cos, i = [], data.find(BUNDLE_MAGIC)
    while i >= 0:
        (n,) = struct.unpack_from("<Q", data, i + len(BUNDLE_MAGIC))
        p = i + len(BUNDLE_MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple.endswith("--" + arch) and size:
                cos.append(data[i + off:i + off + size])
        i = data.find(BUNDLE_MAGIC, i + 1)
    return cos


def _elf_functions(co):
    """(name, machine code bytes) of every FUNC symbol of one ELF64 code object"""
    (shoff,) = struct.unpack_from("<Q", co, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", co, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", co, shoff + k * shentsize) for k in range(shnum)]
    out = []
    for sec in secs:
        if sec[1] != 2:                      # SHT_SYMTAB
            continue
        strtab = secs[sec[6]]
        for k in range(sec[5] // 24):        # Elf64_Sym: name, info, other, shndx, value, size
            name_off, info, _, shndx, value, size = struct.unpack_from("<IBBHQQ", co, sec[4] + 24 * k)
            if info & 0xF != 2 or not size or shndx >= len(secs):   # STT_FUNC with code
                continue
            end = co.index(b"\0", strtab[4] + name_off)
            name = co[strtab[4] + name_off:end].decode()
            text = secs[shndx]
            start = text[4] + (value - text[3])   # file offset = section offset + (address - section address)
            out.append((name, bytes(co[start:start + size])))
    return out


def kernel_code_sha256(so_path, kernels, arch=ARCH):
    """sha256 over the machine code of `kernels` (demangled names as rocprofv3 prints them, e.g.
    "k_seal_uniform<1, true, 0>") in the library's gfx950 code objects: what ties a committed PMC
    count (profiles/pmc_traffic.json) to the build it was measured on -- another kernel's change
    leaves it alone, a change to one of these kernels makes it stale.  None if a kernel is absent."""
    import hashlib
    funcs = [f for co in device_code_objects(so_path, arch) for f in _elf_functions(co)]
    names = [n for n, _ in funcs]
    filt = shutil.which("c++filt") or shutil.which("llvm-cxxfilt")
    dem = subprocess.run([filt], input="\n".join(names), capture_output=True, text=True, check=True).stdout.split("\n")
    code = {}
    for (n, b), d in zip(funcs, dem):
        d = d.replace("(anonymous namespace)::", "")
        code.setdefault(d.split("(")[0].replace("void ", "", 1).strip(), b)
    h = hashlib.sha256()
    for k in sorted(kernels):
        if k not in code:
            return None
        h.update(k.encode() + b"\0" + code[k])
    return h.hexdigest()


def disassemble(code_object, arch=ARCH):
    """llvm-objdump listing of one code object, reduced to instruction lines (no labels or
    encoding comments), the form tools/isa_store_hazard.scan reads."""
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(code_object)
        f.flush()
        out = subprocess.run([os.path.join(LLVM_BIN, "llvm-objdump"), "-d", f"--mcpu={arch}", f.name],
                             check=True, capture_output=True, text=True).stdout
    lines = []
    for ln in out.splitlines():
        ln = ln.split("//")[0].rstrip()
        if ln.strip() and not ln.endswith(":") and not ln.startswith(("Disassembly", "/")):
            lines.append(ln)
    return "\n".join(lines)


def isa_gate(so_path, arch=ARCH):
    """Scan every gfx950 code object of `so_path`; raise IsaHazardError on any hazard.
    Returns (code objects, instructions scanned)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from isa_store_hazard import scan
    cos = device_code_objects(so_path, arch)
    if not cos:
        raise IsaHazardError(f"{so_path}: no {arch} code object found to scan")
    total, hits = 0, []
    for co in cos:
        text = disassemble(co, arch)
        total += text.count("\n") + 1
        d, s, r = scan(text)
        hits += [("store data rewritten at distance 1", x) for x in d]
        hits += [("VALU-written SGPR read by VMEM within 5 states", x) for x in s]
        hits += [("wide buffer store with a register soffset", x) for x in r]
    if hits:
        raise IsaHazardError(f"{so_path}: {len(hits)} VMEM store hazard(s) in the {arch} ISA, "
                             f"library not installed; first: {hits[:3]}")
    return len(cos), total


def build_library(force=False, verbose=True, sources=None, lib=None, src_dir=None, jobs=None):
    """Compile `sources` (default: the product sources in csrc/) in parallel, link `lib`, gate it on
    the ISA scan, then move it into place."""
    sources = list(sources or SOURCES)
    lib = lib or LIB
    src_dir = src_dir or CSRC
    compile_flags(lib)  # refuse product-library builds with extra flags before anything else
    if not force and src_dir == CSRC and not _stale(lib, sources):
        return lib
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    common = compile_flags(lib)
    objdir = tempfile.mkdtemp(prefix="cz_build_")
    try:
        def compile_one(entry):
            f, _, part = entry.partition("#")
            obj = os.path.join(objdir, os.path.splitext(f)[0] + (f"_{part}" if part else "") + ".o")
            cmd = [hipcc] + common + ([f"-DCZ_KPART={part}"] if part else []) + ["-c", "-o", obj, os.path.join(src_dir, f)]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            r = subprocess.run(cmd, cwd=src_dir, capture_output=True, text=True)
            if r.returncode:
                errs = [ln for ln in r.stderr.splitlines() if "error" in ln][:20]
                print("\n".join(errs), file=sys.stderr)
                raise subprocess.CalledProcessError(r.returncode, cmd, r.stdout, r.stderr)
            return obj
        # the largest translation unit first: the kernels dominate the build
        order = sorted(sources, key=lambda f: -os.path.getsize(os.path.join(src_dir, f.split("#")[0])))
        with ThreadPoolExecutor(max_workers=jobs or min(len(order), os.cpu_count() or 4, 8)) as ex:
            objs = list(ex.map(compile_one, order))
        tmp = f"{lib}.{os.getpid()}.tmp"  # (concurrent builds, e.g. pytest -n, never share a file)
        subprocess.check_call([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs, cwd=src_dir)
        try:
            n_co, n_ins = isa_gate(tmp)
        except Exception:
            os.unlink(tmp)
            raise
        if verbose:
            print(f"isa gate: {n_co} {ARCH} code objects, {n_ins} instructions, 0 store hazards", file=sys.stderr)
        os.replace(tmp, lib)
    finally:
        shutil.rmtree(objdir, ignore_errors=True)
    return lib


JNI_DIR = os.path.join(ROOT, "jni")
JNI_BENCH = os.path.join(ROOT, "tools", "bin", "jni_bench")
# the library entry points jni/fake_jni_env.c interposes (tests/test_jni_shim.py links the same list)
JNI_WRAPPED = ("cz_box_afternm", "cz_box_open_afternm", "cz_secretbox", "cz_secretbox_open", "cz_box_beforenm", "cz_box",
               "cz_box_open", "cz_box_keypair", "cz_engine_add_conn")


def build_jni_bench(lib=PRODUCT_LIB, out=JNI_BENCH):
    """tools/bin/jni_bench (bench.py --config jni): the JNI shim, the fake JNIEnv and the driver
    jni/jni_bench.c against the product library, with an $ORIGIN-relative rpath so the binary runs
    from the repository copy on the GPU box."""
    os.makedirs(os.path.dirname(out), exist_ok=True)
    rel = os.path.relpath(os.path.dirname(lib), os.path.dirname(out))
    cmd = ["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror", "-DCZ_JNI_MIN", "-I" + JNI_DIR,
           "-I" + os.path.join(ROOT, "include"), os.path.join(JNI_DIR, "jni_bench.c"),
           os.path.join(JNI_DIR, "curvezmq_jni.c"), os.path.join(JNI_DIR, "fake_jni_env.c"),
           "-L" + os.path.dirname(lib), "-lcurvezmq_mi355x", "-Wl,-rpath,$ORIGIN/" + rel,
           "-Wl," + ",".join("--wrap=" + f for f in JNI_WRAPPED), "-o", out]
    subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    build_library(force="--force" in sys.argv)
    print(LIB)
