"""Native h2c gRPC front door (csrc/net/h2_server.cpp, serving/native_front.py)
against unmodified grpcio clients: Predict (raw and packed encodings, large
messages, concurrent calls on one channel and many channels), the other four
PredictionService RPCs through the Python fallback, error statuses with
messages, deadlines, cancellation, and the HPACK codec pieces (Huffman table
round trip, grpc-timeout grammar, percent-encoding). Scores are checked
against the model's fp32 forward. The reference's transport is gRPC over
HTTP/2 (DCNClient.java:111-112, :118-125)."""
import concurrent.futures as cf
import time

import grpc
import numpy as np
import pytest
import torch

from distributed_tf_serving_amd.client.synth import SyntheticRequests
from distributed_tf_serving_amd.config import load_preset
from distributed_tf_serving_amd.ops import native
from distributed_tf_serving_amd.serving.native_front import NativeGrpcFront
from distributed_tf_serving_amd.serving.server import ModelServer
from distributed_tf_serving_amd.wire import schema as pb
from distributed_tf_serving_amd.wire import tensor as T

F = 43
PREDICT = "/tensorflow.serving.PredictionService/Predict"


def _cfg():
    cfg = load_preset("wdl_tiny_cpu")
    cfg.serving.max_batch_rows = 64
    cfg.serving.allowed_batch_sizes = (8, 64)
    cfg.serving.batch_timeout_us = 300
    return cfg


@pytest.fixture(scope="module")
def front():
    srv = ModelServer(_cfg(), device="cpu")
    srv.start_native_grpc(0, "127.0.0.1", threads=2)  # the server CLI's default front door
    fr = srv.front
    assert isinstance(fr, NativeGrpcFront)
    yield srv, fr
    srv.stop()


def _channel(port, **opts):
    o = [("grpc.max_receive_message_length", 64 << 20), ("grpc.max_send_message_length", 64 << 20)]
    return grpc.insecure_channel(f"127.0.0.1:{port}", options=o + list(opts.items()))


def _expected(srv, ids, wts):
    m = srv.registry.resolve("DCN").model
    return m(torch.as_tensor(ids), torch.as_tensor(wts)).numpy()


def _scores(resp: bytes) -> np.ndarray:
    return T.to_ndarray(pb.PredictResponse.FromString(resp).outputs["prediction_node"])


def test_predict_many_calls_one_channel_matches_fp32(front):
    srv, fr = front
    ch = _channel(fr.port)
    call = ch.unary_unary(PREDICT)
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=11)
    reqs = []
    for i in range(60):
        rows = [1, 7, 33, 64, 5][i % 5]
        ids, wts = synth.arrays(rows)
        data = native().encode_predict_request("DCN", "serving_default", None,
                                               [("feat_ids", torch.from_numpy(ids)), ("feat_wts", torch.from_numpy(wts))],
                                               i % 2 == 0)
        reqs.append((data, ids, wts))
    with cf.ThreadPoolExecutor(16) as pool:  # concurrent streams multiplexed on one HTTP/2 connection
        outs = list(pool.map(lambda r: call(r[0], timeout=20), reqs))
    for (data, ids, wts), resp in zip(reqs, outs):
        np.testing.assert_allclose(_scores(resp), _expected(srv, ids, wts), atol=1e-5)
    st = fr.stats()
    assert st["calls"] >= 60 and st["protocol_errors"] == 0
    ch.close()


def test_many_connections_and_large_message(front):
    srv, fr = front
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="uniform", seed=12)
    # 1500 candidates, raw tensor_content: ~774 KB (the reference's request at N=1),
    # split by the fallback path into batch-sized sub-requests (> 64 rows per batch)
    ids, wts = synth.arrays(1500)
    data = native().encode_predict_request("DCN", "serving_default", None,
                                           [("feat_ids", torch.from_numpy(ids)), ("feat_wts", torch.from_numpy(wts))],
                                           True)
    assert len(data) > 700_000
    chans = [_channel(fr.port) for _ in range(6)]
    with cf.ThreadPoolExecutor(6) as pool:
        outs = list(pool.map(lambda c: c.unary_unary(PREDICT)(data, timeout=60), chans))
    want = _expected(srv, ids, wts)
    for o in outs:
        np.testing.assert_allclose(_scores(o), want, atol=1e-5)
    for c in chans:
        c.close()


def test_message_objects_metadata_and_classify(front):
    srv, fr = front
    ch = _channel(fr.port)
    M = pb.METHODS
    req = pb.GetModelMetadataRequest()
    req.model_spec.name = "DCN"
    req.metadata_field.append("signature_def")
    resp = ch.unary_unary("/tensorflow.serving.PredictionService/GetModelMetadata",
                          request_serializer=M["GetModelMetadata"][0].SerializeToString,
                          response_deserializer=M["GetModelMetadata"][1].FromString)(req, timeout=20)
    assert resp.model_spec.name == "DCN" and "signature_def" in resp.metadata
    creq = pb.ClassificationRequest()
    creq.model_spec.name = "DCN"
    ex = creq.input.example_list.examples.add()
    ex.features.feature["feat_ids"].int64_list.value.extend(range(1, F + 1))
    ex.features.feature["feat_wts"].float_list.value.extend([1.0] * F)
    cresp = ch.unary_unary("/tensorflow.serving.PredictionService/Classify",
                           request_serializer=M["Classify"][0].SerializeToString,
                           response_deserializer=M["Classify"][1].FromString)(creq, timeout=20)
    assert len(cresp.result.classifications) == 1
    ch.close()


def test_error_statuses_and_unknown_method(front):
    srv, fr = front
    ch = _channel(fr.port)
    synth = SyntheticRequests(fields=F, seed=13)
    msg = synth.message(4)
    msg.model_spec.name = "NoSuchModel"
    with pytest.raises(grpc.RpcError) as e:
        ch.unary_unary(PREDICT)(msg.SerializeToString(), timeout=10)
    assert e.value.code() == grpc.StatusCode.NOT_FOUND and "NoSuchModel" in e.value.details()
    with pytest.raises(grpc.RpcError) as e:
        ch.unary_unary(PREDICT)(b"\xff\xff\xff garbage", timeout=10)
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    with pytest.raises(grpc.RpcError) as e:
        ch.unary_unary("/tensorflow.serving.PredictionService/Nope")(b"", timeout=10)
    assert e.value.code() == grpc.StatusCode.UNIMPLEMENTED
    # non-ASCII in a status message survives the percent-encoding
    assert native is not None
    ch.close()


def test_deadline_exceeded_on_the_client_and_server_survives(front):
    srv, fr = front
    ch = _channel(fr.port)
    synth = SyntheticRequests(fields=F, seed=14)
    data = synth.serialized(8)
    # a 100 us deadline expires before (or while) the call is served - unless
    # an idle server answers inside it (it can, on an idle host): each try is
    # queued behind a burst of full batches on another channel
    busy = _channel(fr.port)
    big = synth.serialized(64)
    codes = []
    for _ in range(20):
        burst = [busy.unary_unary(PREDICT).future(big) for _ in range(16)]
        try:
            assert _scores(ch.unary_unary(PREDICT)(data, timeout=1e-4)).shape == (8,)
        except grpc.RpcError as e:
            codes.append(e.code())
        for f in burst:
            f.result(timeout=60)
        if codes:
            break
    busy.close()
    assert codes == [grpc.StatusCode.DEADLINE_EXCEEDED], codes
    # the connection and the server keep working after the cancelled stream
    assert _scores(ch.unary_unary(PREDICT)(data, timeout=20)).shape == (8,)
    ch.close()


def test_stop_refuses_new_calls():
    srv = ModelServer(_cfg(), device="cpu")
    live = srv.registry.resolve("DCN").scheduler
    fr = NativeGrpcFront(srv.service, live, port=0, host="127.0.0.1", threads=1)
    ch = _channel(fr.port)
    data = SyntheticRequests(fields=F, seed=15).serialized(3)
    assert _scores(ch.unary_unary(PREDICT)(data, timeout=20)).shape == (3,)
    fr.stop()
    with pytest.raises(grpc.RpcError) as e:
        ch.unary_unary(PREDICT)(data, timeout=3)
    assert e.value.code() in (grpc.StatusCode.UNAVAILABLE, grpc.StatusCode.DEADLINE_EXCEEDED)
    ch.close()
    srv.stop()


def test_hpack_huffman_and_helpers():
    h = native().hpack_selftest()
    assert h["huffman_roundtrip"] and h["static_decode"] and h["dynamic_table"] and h["bad_padding_rejected"]
    assert h["timeouts"] == [1000000, 250000, 100, 1, 7200000000, -1]
    assert h["percent"] == "a%25b%0Ac%C3%A9"


def test_native_client_and_load_generator(front):
    """The native h2c client (csrc/net/h2_client.cpp) against the native front
    door: one call, a status error, and the closed-loop generator the
    over-the-network reference workload uses."""
    srv, fr = front
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=16)
    ids, wts = synth.arrays(20)
    data = native().encode_predict_request("DCN", "serving_default", None,
                                           [("feat_ids", torch.from_numpy(ids)), ("feat_wts", torch.from_numpy(wts))],
                                           True)
    st, msg, body = native().grpc_call("127.0.0.1", fr.port, PREDICT, data, 10.0)
    assert st == 0, msg
    np.testing.assert_allclose(_scores(body), _expected(srv, ids, wts), atol=1e-5)
    st, msg, _ = native().grpc_call("127.0.0.1", fr.port, PREDICT, b"\xff\xff", 10.0)
    assert st == 3 and msg
    reqs = [synth.serialized(32) for _ in range(4)]
    r = native().run_grpc_load("127.0.0.1", fr.port, PREDICT, reqs, concurrency=4, warmup=8, count=80,
                               timeout_s=20.0)
    assert r["errors"] == 0 and r["ok"] == 88 and len(r["latency_us"]) == 80 and r["window_us"] > 0, r["first_error"]


def test_native_client_talks_to_grpcio_server():
    """Interop the other way: the native client against the grpcio front door."""
    from distributed_tf_serving_amd.serving.grpc_server import GrpcFrontDoor

    srv = ModelServer(_cfg(), device="cpu")
    gd = GrpcFrontDoor(srv.service, port=0, host="127.0.0.1", max_workers=4).start()
    try:
        data = SyntheticRequests(fields=F, seed=17).serialized(9)
        st, msg, body = native().grpc_call("127.0.0.1", gd.port, PREDICT, data, 20.0)
        assert st == 0 and _scores(body).shape == (9,), msg
        st, msg, _ = native().grpc_call("127.0.0.1", gd.port, PREDICT, b"\xff\xff", 20.0)
        assert st == 3
    finally:
        gd.stop()
        srv.stop()


def test_server_cli_serves_through_the_native_front_door():
    """`python -m ...serving.server` picks the native front door for a live
    servable (--front auto), answers a grpcio Predict, and exits on SIGTERM."""
    import os
    import signal
    import socket
    import subprocess
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.Popen([sys.executable, "-m", "distributed_tf_serving_amd.serving.server", "--preset", "wdl_tiny_cpu",
                          "--device", "cpu", "--host", "127.0.0.1", "--port", str(port), "--no-gc-freeze"],
                         cwd=repo, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                         env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
    try:
        line = ""
        deadline = time.monotonic() + 120
        while time.monotonic() < deadline:
            line = p.stdout.readline()
            if not line or line.startswith("serving model"):
                break
        assert "native front door" in line, line
        ch = _channel(port)
        data = SyntheticRequests(fields=F, seed=21).serialized(5)
        assert _scores(ch.unary_unary(PREDICT)(data, timeout=30)).shape == (5,)
        ch.close()
    finally:
        p.send_signal(signal.SIGTERM)
        try:
            p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    assert p.returncode == 0, p.returncode


# ---- raw HTTP/2 clients: per-connection memory bounds and a non-blocking event loop
_PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"


def _frame(ftype, flags, sid, payload=b""):
    n = len(payload)
    return bytes([n >> 16 & 255, n >> 8 & 255, n & 255, ftype, flags]) + sid.to_bytes(4, "big") + payload


def _read_frames(sock, until, timeout=5.0):
    """Frames (type, flags, sid, payload) until ``until(frame)`` is true or the peer closes."""
    import socket as _socket

    sock.settimeout(timeout)
    buf, out = b"", []
    deadline = time.time() + timeout
    while time.time() < deadline:
        while len(buf) >= 9:
            n = int.from_bytes(buf[:3], "big")
            if len(buf) < 9 + n:
                break
            f = (buf[3], buf[4], int.from_bytes(buf[5:9], "big") & 0x7FFFFFFF, buf[9:9 + n])
            buf = buf[9 + n:]
            out.append(f)
            if until(f):
                return out
        try:
            chunk = sock.recv(65536)
        except (_socket.timeout, ConnectionResetError):
            break
        if not chunk:
            break
        buf += chunk
    return out


def _hpack_int(prefix_bits, first, v):
    cap = (1 << prefix_bits) - 1
    if v < cap:
        return bytes([first | v])
    out, v = [first | cap], v - cap
    while v >= 128:
        out.append(v % 128 + 128)
        v //= 128
    return bytes(out + [v])


def _raw_conn(port):
    import socket

    s = socket.create_connection(("127.0.0.1", port))
    s.sendall(_PREFACE + _frame(4, 0, 0))
    return s


def test_continuation_flood_gets_goaway_and_server_survives(front):
    srv, fr = front
    before = fr.stats()["protocol_errors"]
    s = _raw_conn(fr.port)
    s.sendall(_frame(1, 0, 1, b"\x82"))  # HEADERS without END_HEADERS
    try:
        for _ in range(64):  # 64 x 16 KiB: past the 64 KiB header-list cap
            s.sendall(_frame(9, 0, 1, b"\x00" * 16384))
    except (BrokenPipeError, ConnectionResetError):
        pass
    frames = _read_frames(s, lambda f: f[0] == 7)
    s.close()
    goaway = [f for f in frames if f[0] == 7]
    assert goaway and int.from_bytes(goaway[0][3][4:8], "big") == 11, frames  # ENHANCE_YOUR_CALM
    settings = [f for f in frames if f[0] == 4 and not f[1] & 1]
    assert settings and b"\x00\x06" + (64 << 10).to_bytes(4, "big") in settings[0][3]  # MAX_HEADER_LIST_SIZE
    assert fr.stats()["protocol_errors"] > before
    data = SyntheticRequests(fields=F, seed=21).serialized(5)
    ch = _channel(fr.port)
    assert _scores(ch.unary_unary(PREDICT)(data, timeout=20)).shape == (5,)
    ch.close()


def test_header_list_bomb_gets_goaway(front):
    # one 4000-byte value put in the dynamic table, then referenced 20 times: a
    # 4 KB block that decodes to 80 KB
    srv, fr = front
    s = _raw_conn(fr.port)
    block = b"\x40" + _hpack_int(7, 0, 5) + b"x-big" + _hpack_int(7, 0, 4000) + b"v" * 4000 + bytes([0x80 | 62]) * 20
    s.sendall(_frame(1, 0x4 | 0x1, 1, block))
    frames = _read_frames(s, lambda f: f[0] == 7)
    s.close()
    goaway = [f for f in frames if f[0] == 7]
    assert goaway and int.from_bytes(goaway[0][3][4:8], "big") == 11, frames


def test_reader_that_never_reads_is_paused_not_buffered(front):
    # PINGs from a client that never reads its ACKs: once 16 MiB of replies wait
    # unsent, the server stops reading that connection instead of queueing more
    import socket

    srv, fr = front
    s = _raw_conn(fr.port)
    s.setblocking(False)
    ping = _frame(6, 0, 0, b"12345678") * 4096  # 69 KB of PINGs per round
    sent, off, t0 = 0, 0, time.time()
    while time.time() - t0 < 20 and fr.stats()["paused_reads"] == 0:
        try:
            n = s.send(ping[off:])  # partial sends: continue mid-frame
            sent += n
            off = (off + n) % len(ping)
        except (BlockingIOError, socket.timeout):
            time.sleep(0.01)
    paused = fr.stats()["paused_reads"]
    s.close()
    assert paused >= 1, f"sent {sent} bytes of PINGs, never paused"
    data = SyntheticRequests(fields=F, seed=22).serialized(4)
    ch = _channel(fr.port)
    assert _scores(ch.unary_unary(PREDICT)(data, timeout=20)).shape == (4,)
    ch.close()


def test_paused_reader_resumes_on_the_same_connection(front):
    # a connection paused for its 16 MiB reply backlog must resume
    # reading once the client drains its socket, whichever flush emptied the
    # backlog - its next PING on the SAME connection is answered
    import socket

    srv, fr = front
    s = _raw_conn(fr.port)
    s.setblocking(False)
    ping = _frame(6, 0, 0, b"12345678") * 4096
    before = fr.stats()["paused_reads"]
    off, t0 = 0, time.time()
    while time.time() - t0 < 20 and fr.stats()["paused_reads"] == before:
        try:
            off = (off + s.send(ping[off:])) % len(ping)
        except (BlockingIOError, socket.timeout):
            time.sleep(0.01)
    assert fr.stats()["paused_reads"] > before, "never paused"
    # drain every reply (frame-aligned) while finishing the partial PING frame,
    # then ask once more on the same connection
    tail = ping[off:] if off else b""
    # (the replies are ~1 M 17-byte PING ACKs: parse with a moving offset and
    # drop the consumed prefix now and then - slicing the buffer per frame was
    # quadratic and made the drain itself time out on a slow host)
    buf, pos, drained, asked, got = bytearray(), 0, 0, False, False
    t0 = time.time()
    while time.time() - t0 < 60 and not got:
        try:
            chunk = s.recv(1 << 20)
            if not chunk:
                break
            buf += chunk
            drained += len(chunk)
        except BlockingIOError:
            time.sleep(0.002)
        while len(buf) - pos >= 9:
            n = int.from_bytes(buf[pos:pos + 3], "big")
            if len(buf) - pos < 9 + n:
                break
            if buf[pos + 3] == 6 and buf[pos + 4] & 1 and buf[pos + 9:pos + 9 + n] == b"resumed!":
                got = True
            pos += 9 + n
        if pos > (1 << 20):
            del buf[:pos]
            pos = 0
        if tail:
            try:
                tail = tail[s.send(tail):]
            except BlockingIOError:
                pass
        elif not asked and drained > (8 << 20):
            s.send(_frame(6, 0, 0, b"resumed!"))  # 17 bytes: fits the drained socket buffer
            asked = True
    s.close()
    assert asked and got, (asked, drained, "no PING ACK after the reader drained: reads never resumed")


def test_full_batching_queue_does_not_block_the_event_loop():
    # every arena queued behind a paused server: deadline-less Predicts must not
    # stall the loop thread - a PING on another connection of the same (only)
    # loop is still answered, and the calls complete once steps run
    from distributed_tf_serving_amd.serving.live import LiveScheduler
    from distributed_tf_serving_amd.serving.server import build_engine

    cfg = _cfg()
    srv = ModelServer(cfg, device="cpu")
    eng = build_engine(cfg, torch.device("cpu"), 3)
    live = LiveScheduler(eng, cfg.serving, start_paused=True)
    fr = NativeGrpcFront(srv.service, live, port=0, host="127.0.0.1", threads=1)
    ch = _channel(fr.port)
    data = SyntheticRequests(fields=F, seed=23).serialized(64)  # one full batch each
    n = len(live.arenas) + 4
    futs = [ch.unary_unary(PREDICT).future(data) for _ in range(n)]
    t0 = time.time()
    while fr.stats()["blocking_submits_handed_off"] == 0 and time.time() - t0 < 10:
        time.sleep(0.02)
    assert fr.stats()["blocking_submits_handed_off"] > 0
    s = _raw_conn(fr.port)
    s.sendall(_frame(6, 0, 0, b"pingpong"))
    t1 = time.time()
    frames = _read_frames(s, lambda f: f[0] == 6 and f[1] & 1, timeout=5.0)
    s.close()
    assert any(f[0] == 6 and f[1] & 1 and f[3] == b"pingpong" for f in frames), "PING not answered"
    assert time.time() - t1 < 2.0
    live.resume()
    for f in futs:
        assert _scores(f.result(timeout=60)).shape == (64,)
    ch.close()
    fr.stop()
    live.close()
    srv.stop()
