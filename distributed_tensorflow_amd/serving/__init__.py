"""REST model server for exported SavedModels.

Replaces the external ``simple_tensorflow_serving --port=8500 --model_base_path=./saved_model``
of the reference runbook (reference README.md:29-41). Accepts the README's request verbatim:

    POST /  {"keys": [[11.0], [2.0]], "features": [[1], [2]]}

(the README sends ``keys`` as floats and ``features`` as ints, i.e. swapped relative to the
signature's int32 / float32: inputs are coerced to the signature dtypes), plus the
simple_tensorflow_serving envelope ``{"model_name", "model_version", "signature_name", "data": {...}}``
and TF-Serving's ``POST /v1/models/<name>:predict {"inputs": {...}}`` / ``{"instances": [...]}``.
Responses are JSON of every signature output. ``GET /`` and ``/v1/models/<name>`` report status.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import torch

from .. import saved_model


class ModelServer:
    def __init__(self, model_base_path, model_name="default", device=None):
        self.base = model_base_path
        self.name = model_name
        self.version_dir = saved_model.latest_version_dir(model_base_path)
        self.version = os.path.basename(self.version_dir.rstrip("/"))
        self.loaded = saved_model.load(self.version_dir, device=device)
        self._lock = threading.Lock()
        self.requests = 0

    def predict(self, body):
        sig_name = body.get("signature_name") or saved_model.DEFAULT_SERVING_SIGNATURE_DEF_KEY
        sig = self.loaded.signatures[sig_name]
        if "data" in body and isinstance(body["data"], dict):
            inputs = body["data"]
        elif "inputs" in body and isinstance(body["inputs"], dict):
            inputs = body["inputs"]
        elif "instances" in body:
            inst = body["instances"]
            inputs = {k: [row[k] for row in inst] for k in sig.structured_input_signature} if inst and isinstance(
                inst[0], dict) else {next(iter(sig.structured_input_signature)): inst}
        else:
            inputs = {k: v for k, v in body.items() if k in sig.structured_input_signature}
        with self._lock:
            out = sig(**inputs)
            self.requests += 1
        return {k: (v.detach().cpu().tolist() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}

    def status(self):
        return {"model_name": self.name, "model_version": self.version, "path": self.version_dir,
                "signatures": {k: {"inputs": s.structured_input_signature, "outputs": s.structured_outputs}
                               for k, s in self.loaded.signatures.items()}}


def make_handler(server):
    class Handler(BaseHTTPRequestHandler):
        def _send(self, code, obj):
            b = json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(b)))
            self.end_headers()
            self.wfile.write(b)

        def do_GET(self):
            self._send(200, server.status())

        def do_POST(self):
            try:
                n = int(self.headers.get("Content-Length", "0"))
                body = json.loads(self.rfile.read(n) or b"{}")
                res = server.predict(body)
                if self.path.startswith("/v1/models/"):
                    res = {"outputs": res}
                self._send(200, res)
            except Exception as e:
                self._send(400, {"error": f"{type(e).__name__}: {e}"})

        def log_message(self, *a):
            pass
    return Handler


def serve(model_base_path, port=8500, host="0.0.0.0", model_name="default", device=None, block=True):
    ms = ModelServer(model_base_path, model_name, device)
    httpd = ThreadingHTTPServer((host, port), make_handler(ms))
    if not block:
        th = threading.Thread(target=httpd.serve_forever, daemon=True)
        th.start()
        return httpd, ms
    print(f"serving {ms.version_dir} on {host}:{httpd.server_address[1]}", flush=True)
    try:
        httpd.serve_forever()
    except KeyboardInterrupt:
        pass
    return httpd, ms


def main(argv=None):
    ap = argparse.ArgumentParser("dtf-serve")
    ap.add_argument("--port", type=int, default=8500)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--model_base_path", default="./saved_model")
    ap.add_argument("--model_name", default="default")
    a = ap.parse_args(argv)
    serve(a.model_base_path, a.port, a.host, a.model_name)
    return 0


if __name__ == "__main__":
    sys.exit(main())
