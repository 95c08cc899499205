"""Codegen check of the bench kernels' tile loops in the built library (no GPU needed).

A tile loop loads the next tile's input (the RX's window slots, the TX's bits words) while it stores
the current tile's outputs. Vector-memory counters retire in issue order, so the wait for a slot's
load only has to leave the stores issued after it in flight: vmcnt(N) with N >= the stores of one
trip. Round 5 found the compiler waiting for all of them instead (vmcnt(0..7)) wherever a store sat
under a runtime branch in the loop, a loop exit shared the latch, a load was left pending on entry,
or the stores were flat (profiles/r05_waitcnt.txt) -- every tile then waited for the previous tile's
stores to complete. This reads each kernel's disassembly from lib/libmodem_hip.so and asserts that
every tile loop's waits leave a trip's stores in flight.
"""
import os
import re
import shutil
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "rust-modem_amd", "lib", "libmodem_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"

KERNELS = {
    "c3 rx": "_ZN2mk7rx_mfmaILi4ELi6EfLi0EfLi4ELi3ELi1EEEvNS_8RxParamsEPKDF16_i",
    "c3 tx": "_ZN2mk7tx_mfmaILi4ELi2ELi0EfLi4EEEvNS_8TxParamsEPKDv8_DF16_i",
    "c4 rx batch": "_ZN2mk13rx_mfma_batchILi4ELi4EfLi0EfLi4ELi7ELi1EEEvNS_7RxBatchEPKDF16_",
    "c4 tx batch": "_ZN2mk13tx_mfma_batchILi4ELi1ELi0EfLi4EEEvNS_7TxBatchEPKDv8_DF16_",
    "c5 rx (k-split)": "_ZN2mk7rx_mfmaILi8ELi20EfLi0EfLi4ELi3ELi2EEEvNS_8RxParamsEPKDF16_i",
    "c5 tx": "_ZN2mk7tx_mfmaILi8ELi3ELi0EfLi4EEEvNS_8TxParamsEPKDv8_DF16_i",
    "c5 f16 rx": "_ZN2mk7rx_mfmaILi8ELi20E6__halfLi0ES1_Li4ELi3ELi1EEEvNS_8RxParamsEPKDF16_i",
    "c5 f16 tx": "_ZN2mk7tx_mfmaILi8ELi3ELi0E6__halfLi4EEEvNS_8TxParamsEPKDv8_DF16_i",
}


def _tools_ok():
    return (os.path.exists(LIB) and shutil.which("objcopy")
            and all(os.path.exists(os.path.join(LLVM, t)) for t in ("llvm-objdump", "llvm-readelf")))


@pytest.fixture(scope="module")
def code_objects(tmp_path_factory):
    if not _tools_ok():
        pytest.skip("library or binutils / llvm tools missing")
    d = tmp_path_factory.mktemp("isa")
    fb = d / "fatbin"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", LIB, str(fb)], check=True)
    data = fb.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    objs = []
    i = data.find(magic)
    while i != -1:                          # clang offload bundles: magic, count, (offset, size, triple)*
        p = i + len(magic)
        n = struct.unpack_from("<Q", data, p)[0]
        p += 8
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            if "gfx950" in triple:
                f = d / f"co{len(objs)}.o"
                f.write_bytes(data[i + off:i + off + size])
                symtab = subprocess.run([f"{LLVM}/llvm-readelf", "-sW", str(f)], capture_output=True, text=True).stdout
                objs.append((str(f), symtab))
        i = data.find(magic, i + 1)
    assert objs, "no gfx950 code object in the library"
    return objs


def _disassemble(objs, name):
    for f, symtab in objs:
        for line in symtab.split("\n"):
            t = line.split()
            if len(t) >= 8 and t[7] == name and t[3] == "FUNC":
                st, sz = int(t[1], 16), int(t[2])
                return subprocess.run([f"{LLVM}/llvm-objdump", "-d", f"--start-address={st}", f"--stop-address={st + sz}", f],
                                      capture_output=True, text=True).stdout
    return None


def tile_loops(dis):
    """(stores, loads, min vmcnt) of every loop -- a backward branch to a label -- whose body holds one
    trip of a tile loop: 4..12 vector-memory loads (one tile's slots or bits words) and >= 8 stores."""
    ins = []                                   # (mnemonic, operands, address)
    for line in dis.split("\n"):
        m = re.match(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):", line)
        if m:
            ins.append((m.group(1), m.group(2), int(m.group(3), 16)))
    at = {addr: k for k, (_, _, addr) in enumerate(ins)}
    out = []
    for k, (o, a, addr) in enumerate(ins):
        if not (o.startswith("s_cbranch") or o == "s_branch") or not re.fullmatch(r"\d+", a):
            continue
        simm = int(a) & 0xFFFF                 # SOPP branch: target = next instruction + 4 * simm16
        tgt = at.get(addr + 4 + 4 * ((simm ^ 0x8000) - 0x8000))
        if tgt is None or tgt >= k:
            continue
        body = ins[tgt:k + 1]
        vmem = [x for x, _, _ in body if not x.startswith(("ds_", "s_"))]
        stores = sum(1 for x in vmem if "_store" in x)
        loads = sum(1 for x in vmem if "_load" in x)
        waits = [int(re.search(r"vmcnt\((\d+)\)", y).group(1)) for x, y, _ in body if x == "s_waitcnt" and "vmcnt" in y]
        if stores >= 8 and 4 <= loads <= 12:
            out.append((stores, loads, min(waits) if waits else None))
    return out


@pytest.mark.parametrize("what", sorted(KERNELS))
def test_tile_loop_waits_leave_the_stores_in_flight(code_objects, what):
    dis = _disassemble(code_objects, KERNELS[what])
    assert dis, f"{what}: kernel {KERNELS[what]} not in the library"
    loops = tile_loops(dis)
    assert loops, f"{what}: no tile loop found"
    for stores, loads, w in loops:
        assert w is None or w >= stores, (f"{what}: a tile loop ({loads} loads, {stores} stores per trip) waits "
                                          f"vmcnt({w}), i.e. for the trip's stores")
