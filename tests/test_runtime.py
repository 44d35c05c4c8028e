"""Native runtime (CPU): CRC32C, tensor-bundle checkpoints (cross-checked with the protobuf library),
TFRecord/event files, KV store, shared-memory all-reduce, PS transport."""
import multiprocessing as mp
import os
import struct
import threading

import numpy as np
import pytest
import torch

from distributed_tensorflow_amd import _native


def test_crc32c_known_values():
    lib = _native.runtime()
    assert lib.dtfrt_crc32c(b"123456789", 9, 0) == 0xE3069283
    assert lib.dtfrt_crc32c(b"", 0, 0) == 0
    data = os.urandom(10007)
    a = lib.dtfrt_crc32c(data, len(data), 0)
    b = lib.dtfrt_crc32c(data[5000:], len(data) - 5000, lib.dtfrt_crc32c(data, 5000, 0))
    assert a == b


def test_bundle_roundtrip_dtypes_shards_and_checksums(tmp_path):
    from distributed_tensorflow_amd.train import checkpoint as C
    tens = {"a/f32": torch.randn(3, 5), "b/bf16": torch.randn(7).to(torch.bfloat16),
            "c/i64": torch.arange(10, dtype=torch.int64), "d/scalar": torch.tensor(3.5),
            "e/big": torch.randn(300, 257), "meta": "json-ish string"}
    for i in range(40):  # enough keys to span several restart intervals
        tens[f"layer_{i:03d}/kernel"] = torch.randn(4, 4)
    p = C.save_tensors(str(tmp_path / "ck"), tens, num_shards=3, shard_of=lambda k, i: i % 3)
    out = C.load_tensors(p)
    assert set(out) == set(tens)
    for k, v in tens.items():
        if isinstance(v, str):
            assert out[k] == v.encode()
        else:
            assert out[k].dtype == v.dtype and torch.equal(out[k], v)
    # corruption of a data shard is detected by the per-entry CRC
    shard = [f for f in os.listdir(tmp_path) if ".data-00001-of-00003" in f][0]
    raw = bytearray(open(tmp_path / shard, "rb").read())
    raw[len(raw) // 2] ^= 0xFF
    open(tmp_path / shard, "wb").write(bytes(raw))
    r = C.BundleReader(p)
    bad = 0
    for k in r.names():
        try:
            r.read(k)
        except IOError:
            bad += 1
    assert bad == 1


def _proto_classes():
    """Build BundleEntryProto / BundleHeaderProto / TensorShapeProto with the protobuf runtime."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    fdp = descriptor_pb2.FileDescriptorProto(name="dtf_test_bundle.proto", package="tftest", syntax="proto3")
    dim = fdp.message_type.add(name="Dim")
    dim.field.add(name="size", number=1, type=3, label=1)
    shp = fdp.message_type.add(name="TensorShapeProto")
    shp.field.add(name="dim", number=2, type=11, label=3, type_name=".tftest.Dim")
    ver = fdp.message_type.add(name="VersionDef")
    ver.field.add(name="producer", number=1, type=5, label=1)
    hdr = fdp.message_type.add(name="BundleHeaderProto")
    hdr.field.add(name="num_shards", number=1, type=5, label=1)
    hdr.field.add(name="endianness", number=2, type=5, label=1)
    hdr.field.add(name="version", number=3, type=11, label=1, type_name=".tftest.VersionDef")
    ent = fdp.message_type.add(name="BundleEntryProto")
    ent.field.add(name="dtype", number=1, type=5, label=1)
    ent.field.add(name="shape", number=2, type=11, label=1, type_name=".tftest.TensorShapeProto")
    ent.field.add(name="shard_id", number=3, type=5, label=1)
    ent.field.add(name="offset", number=4, type=3, label=1)
    ent.field.add(name="size", number=5, type=3, label=1)
    ent.field.add(name="crc32c", number=6, type=7, label=1)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    get = message_factory.GetMessageClass
    return get(pool.FindMessageTypeByName("tftest.BundleHeaderProto")), \
        get(pool.FindMessageTypeByName("tftest.BundleEntryProto"))


def _sstable_entries(path):
    """Independent Python parse of the .index SSTable (footer -> index block -> data blocks)."""
    b = open(path, "rb").read()
    assert struct.unpack("<Q", b[-8:])[0] == 0xDB4775248B80FB57

    def varint(p):
        v, s = 0, 0
        while True:
            c = b[p]
            p += 1
            v |= (c & 0x7F) << s
            s += 7
            if not c & 0x80:
                return v, p
    foot = len(b) - 48
    _, p = varint(foot)
    _, p = varint(p)
    io, p = varint(p)
    isz, p = varint(p)

    def block(off, size):
        blk = b[off:off + size]
        assert b[off + size] == 0  # no compression
        nr = struct.unpack("<I", blk[-4:])[0]
        end = len(blk) - 4 - 4 * nr
        q, key, out = 0, b"", []
        while q < end:
            sh, q2 = varint(off + q)
            ns, q2 = varint(q2)
            vl, q2 = varint(q2)
            q2 -= off
            key = key[:sh] + blk[q2:q2 + ns]
            out.append((key, blk[q2 + ns:q2 + ns + vl]))
            q = q2 + ns + vl
        return out
    entries = []
    for _, h in block(io, isz):
        hb = bytes(h)
        v, q = 0, 0
        vals = []
        for _ in range(2):
            v, s = 0, 0
            while True:
                c = hb[q]
                q += 1
                v |= (c & 0x7F) << s
                s += 7
                if not c & 0x80:
                    break
            vals.append(v)
        entries += block(*vals)
    return entries


def test_bundle_index_is_a_valid_sstable_of_tf_protos(tmp_path):
    from distributed_tensorflow_amd.train import checkpoint as C
    Header, Entry = _proto_classes()
    t = {"weight": torch.randn(2, 3), "bias": torch.tensor(1.0), "global_step": torch.tensor(5, dtype=torch.int64)}
    p = C.save_tensors(str(tmp_path / "m"), t)
    ents = _sstable_entries(p + ".index")
    keys = [k for k, _ in ents]
    assert keys == sorted(keys) and keys[0] == b""
    h = Header()
    h.ParseFromString(ents[0][1])
    assert h.num_shards == 1 and h.version.producer == 1
    e = {k.decode(): Entry.FromString(v) for k, v in ents[1:]}
    assert e["weight"].dtype == 1 and [d.size for d in e["weight"].shape.dim] == [2, 3]
    assert e["weight"].size == 24
    assert e["global_step"].dtype == 9 and list(e["global_step"].shape.dim) == []
    lib = _native.runtime()
    data = open(p + ".data-00000-of-00001", "rb").read()
    ew = e["weight"]
    assert lib.dtfrt_crc_mask(lib.dtfrt_crc32c(data[ew.offset:ew.offset + ew.size], ew.size, 0)) == ew.crc32c


def test_saver_rotation_and_state_file(tmp_path):
    from distributed_tensorflow_amd import Variable
    from distributed_tensorflow_amd.train import checkpoint as C
    v = Variable(torch.zeros(4), name="v")
    s = C.Saver([v], max_to_keep=2)
    for step in range(4):
        v.assign(torch.full((4,), float(step)))
        s.save(None, str(tmp_path / "model.ckpt"), global_step=step)
    st = C.get_checkpoint_state(str(tmp_path))
    assert os.path.basename(st["model_checkpoint_path"]) == "model.ckpt-3"
    assert [os.path.basename(x) for x in st["all_model_checkpoint_paths"]] == ["model.ckpt-2", "model.ckpt-3"]
    assert not (tmp_path / "model.ckpt-0.index").exists()
    v.assign(torch.zeros(4))
    s.restore(None, C.latest_checkpoint(str(tmp_path)))
    assert torch.equal(v.detach(), torch.full((4,), 3.0))


def test_object_checkpoint_model_and_optimizer(tmp_path):
    from distributed_tensorflow_amd.keras import layers, losses, optimizers
    from distributed_tensorflow_amd.keras.models import Sequential
    from distributed_tensorflow_amd.train import Checkpoint, CheckpointManager
    m = Sequential([layers.Dense(8, activation="relu"), layers.Dense(3)])
    m.compile(optimizers.Adam(0.01), losses.SparseCategoricalCrossentropy(from_logits=True))
    x, y = torch.randn(32, 5), torch.randint(0, 3, (32,))
    m.fit(x, y, batch_size=8, epochs=1, verbose=0)
    mgr = CheckpointManager(Checkpoint(model=m, optimizer=m.optimizer), str(tmp_path), max_to_keep=2)
    p = mgr.save()
    w0 = [w.detach().clone() for w in m.weights]
    slot0 = m.optimizer.get_slot(m.trainable_weights[0], "Adam").clone()
    m.fit(x, y, batch_size=8, epochs=1, verbose=0)
    st = Checkpoint(model=m, optimizer=m.optimizer).restore(p)
    st.assert_consumed()
    for a, b in zip(m.weights, w0):
        assert torch.equal(a.detach(), b)
    assert torch.equal(m.optimizer.get_slot(m.trainable_weights[0], "Adam"), slot0)
    assert mgr.latest_checkpoint == p


def test_event_file_records(tmp_path):
    from distributed_tensorflow_amd import summary
    w = summary.FileWriter(str(tmp_path), graph="g")
    for s in range(5):
        w.add_summary({"loss": 1.0 / (s + 1)}, s)
    w.text("note", "hello", 1)
    w.close()
    recs = summary.read_events(w.path)
    assert recs[0][2]["__file_version__"] == "brain.Event:2"
    losses = [(st, v["loss"]) for _, st, v in recs if "loss" in v]
    assert losses == [(s, pytest.approx(1.0 / (s + 1))) for s in range(5)]


def test_tfrecord_detects_corruption(tmp_path):
    lib = _native.runtime()
    p = str(tmp_path / "x.tfrecord").encode()
    h = lib.dtfrt_tfrecord_writer_open(p, 0)
    for i in range(3):
        d = f"record-{i}".encode()
        lib.dtfrt_tfrecord_write(h, d, len(d))
    lib.dtfrt_tfrecord_writer_close(h)
    raw = bytearray(open(p, "rb").read())
    raw[14] ^= 1
    open(p, "wb").write(bytes(raw))
    import ctypes
    r = lib.dtfrt_tfrecord_reader_open(p)
    d, n = ctypes.c_void_p(), ctypes.c_uint64()
    assert lib.dtfrt_tfrecord_next(r, ctypes.addressof(d), ctypes.addressof(n)) < 0
    lib.dtfrt_tfrecord_reader_close(r)


def test_kv_store_blocking_get_counters_barrier():
    from distributed_tensorflow_amd.parallel.kv import KVClient, KVServer
    s = KVServer("127.0.0.1", 0)
    try:
        a = KVClient("127.0.0.1", s.port)
        b = KVClient("127.0.0.1", s.port)
        assert a.get("missing", timeout_s=0.05) is None
        got = {}
        th = threading.Thread(target=lambda: got.setdefault("v", b.get("late")))
        th.start()
        a.set("late", b"value")
        th.join(5)
        assert got["v"] == b"value"
        assert a.add("c", 2) == 2 and b.add("c", 3) == 5
        assert not a.wait_ge("c", 6, timeout_s=0.05)
        b.add("c", 1)
        assert a.wait_ge("c", 6, timeout_s=1)
        a.set("p/x", "1")
        a.set("p/y", "2")
        assert sorted(a.keys("p/")) == ["p/x", "p/y"]
        res = []
        ths = [threading.Thread(target=lambda c=c: res.append(c.barrier("b1", 2, 5))) for c in (a, b)]
        [t.start() for t in ths]
        [t.join(10) for t in ths]
        assert res == [True, True]
    finally:
        s.stop()


def _shm_worker(rank, world, name, q):
    from distributed_tensorflow_amd import _native as N
    lib = N.runtime()
    h = lib.dtfrt_shm_open(name.encode(), rank, world, 1 << 16)
    x = np.full(40000, rank + 1, dtype=np.float32)  # spans several chunks of the 64 KiB slots
    rc = lib.dtfrt_shm_allreduce_f32(h, x.ctypes.data, x.size)
    q.put((rank, rc, float(x[0]), float(x[-1])))
    lib.dtfrt_shm_close(h, 0)


def test_shm_allreduce_two_processes():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"t{os.getpid()}"
    ps = [ctx.Process(target=_shm_worker, args=(r, 3, name, q)) for r in range(3)]
    [p.start() for p in ps]
    [p.join(60) for p in ps]
    out = sorted(q.get(timeout=5) for _ in range(3))
    assert all(rc == 0 and a == 6.0 and b == 6.0 for _, rc, a, b in out)


def test_ps_transport_pull_push_roundtrip():
    import ctypes
    lib = _native.runtime()
    bound = ctypes.c_int()
    srv = lib.dtfrt_ps_server_start(b"127.0.0.1", 0, ctypes.addressof(bound))
    mirror = torch.arange(16, dtype=torch.float32)
    lib.dtfrt_ps_register(srv, 0, mirror.data_ptr(), 64)
    from distributed_tensorflow_amd.parallel.parameter_server import PSClient
    c = PSClient("127.0.0.1", bound.value)
    buf = torch.zeros(16)
    c.pull(0, buf)
    assert torch.equal(buf, mirror)

    def apply():
        v, o, n, d = ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_void_p()
        tok = lib.dtfrt_ps_next_push(srv, 5000, ctypes.addressof(v), ctypes.addressof(o), ctypes.addressof(n),
                                     ctypes.addressof(d))
        g = np.frombuffer((ctypes.c_char * n.value).from_address(d.value), dtype=np.float32).copy()
        lib.dtfrt_ps_lock(srv, 0)
        mirror.sub_(torch.from_numpy(g))
        lib.dtfrt_ps_unlock(srv, 0, 1)
        lib.dtfrt_ps_push_done(srv, tok, 0)
    th = threading.Thread(target=apply)
    th.start()
    ver = c.push(0, torch.ones(16))
    th.join(5)
    assert ver == 1
    c.pull(0, buf)
    assert torch.equal(buf, torch.arange(16, dtype=torch.float32) - 1)
    c.close()
    lib.dtfrt_ps_server_stop(srv)


@pytest.mark.slow
def test_runtime_under_sanitizers(tmp_path):
    """ASan+UBSan and TSan builds of the C++ runtime run a concurrent self-test cleanly."""
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["bash", os.path.join(root, "tools", "sanitize_runtime.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "sanitizers clean" in r.stdout
