#!/usr/bin/env python3
"""BASELINE config 4 throughput: s3:// (and http://) objects -> parallel ranged
GETs -> pinned-host ring -> HIP tile parser -> CSR in HBM, on one GPU.

The objects are served over loopback by tools/dmlc_objserver (sendfile from
the page cache, so the server is not the bound); the same files parsed from
local disk give the reference point.  Each configuration runs one warm epoch
and then --epochs timed epochs of GPUParser.parse_all; the parser's ring
statistics split the time into waiting for the reader (wait_reader_sec: the
network / storage side is the bound) and waiting for the GPU (wait_gpu_sec).
Prints one JSON object.

usage: python scripts/bench_remote.py [--rows N] [--files F] [--epochs E]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--files", type=int, default=8)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--threads", default="8,16,32", help="read_threads values for s3://")
    ap.add_argument("--data", default="/tmp/dmlc_remote_bench")
    ap.add_argument("--reader-threads", default="8,16,32,64",
                    help="read_threads values for the reader-alone runs (tools/dmlc_bench_read)")
    ap.add_argument("--tls", action="store_true",
                    help="serve https (the objserver's --tls) and read s3:// / https:// over it")
    args = ap.parse_args()

    import torch

    from dmlc_core_amd import _dmlc, data

    bucket = os.path.join(args.data, "bench", "train")
    os.makedirs(bucket, exist_ok=True)
    per = args.rows // args.files
    for i in range(args.files):
        f = os.path.join(bucket, f"part-{i:03d}.libsvm")
        if not os.path.exists(f):
            data.write_synthetic(f + ".tmp", i * per, (i + 1) * per, format="libsvm", seed=3,
                                 nthread=16)
            os.replace(f + ".tmp", f)
    nbytes = sum(os.path.getsize(os.path.join(bucket, x)) for x in os.listdir(bucket))
    cmd = [os.path.join(ROOT, "build", "dmlc_objserver"), "--root", args.data]
    scheme = "http"
    if args.tls:
        # https with a self-signed certificate that both the native receive
        # (OpenSSL) and libcurl trust (SSL_CERT_FILE / CURL_CA_BUNDLE): peer
        # and host verified as against a real endpoint
        crt, key = os.path.join(args.data, "tls.crt"), os.path.join(args.data, "tls.key")
        if not os.path.exists(crt):
            subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key,
                            "-out", crt, "-days", "7", "-subj", "/CN=127.0.0.1",
                            "-addext", "subjectAltName=IP:127.0.0.1"], check=True, capture_output=True)
        cmd += ["--tls", crt, key]
        os.environ.update({"SSL_CERT_FILE": crt, "CURL_CA_BUNDLE": crt})
        scheme = "https"
    srv = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    try:
        port = int(srv.stdout.readline().split()[1])
        os.environ.update({"S3_ENDPOINT": f"{scheme}://127.0.0.1:{port}", "S3_ACCESS_KEY_ID": "bench",
                           "S3_SECRET_ACCESS_KEY": "bench", "S3_REGION": "us-east-1"})
        # the host stage alone (ShardReader.Fill into a 64 MiB buffer, no GPU):
        # what the ring's reader can deliver, natively received and via libcurl
        out_reader = []
        for native in ("1", "0"):
            for t in [x for x in args.reader_threads.split(",") if x]:
                env = dict(os.environ, DMLC_HTTP_NATIVE=native)
                p = subprocess.run([os.path.join(ROOT, "build", "dmlc_bench_read"), "s3://bench/train/",
                                    t, "64", str(args.epochs)], capture_output=True, text=True,
                                   env=env, timeout=600)
                rec = json.loads(p.stdout.strip().splitlines()[-1])
                rec["native"] = native == "1"
                out_reader.append(rec)
                print(json.dumps(rec), file=sys.stderr, flush=True)
        runs = [("local", bucket + "/", 8)]
        runs += [("s3", "s3://bench/train/", int(t)) for t in args.threads.split(",") if t]
        runs.append(("http_one_file", f"{scheme}://127.0.0.1:{port}/bench/train/part-000.libsvm", 16))
        out = {"rows": args.rows, "files": args.files, "bytes": nbytes, "epochs": args.epochs,
               "scheme": scheme,
               "server": "tools/dmlc_objserver (loopback, " + ("TLS, pread + SSL_write)" if args.tls
                                                               else "sendfile)"),
               "reader_alone": out_reader,
               "runs": []}
        for name, uri, threads in runs:
            gp = data.GPUParser(uri, format="libsvm", read_threads=threads)
            csr = data.DeviceCSR()
            gp.parse_all(csr)  # warm epoch: page cache, pinned ring, output reserve
            torch.cuda.synchronize()
            s0 = gp.stats()
            t0 = time.perf_counter()
            rows = 0
            for _ in range(args.epochs):
                gp.before_first()
                csr.clear()
                gp.parse_all(csr)
                rows += csr.rows
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            s1 = gp.stats()
            part = nbytes if name != "http_one_file" else os.path.getsize(
                os.path.join(bucket, "part-000.libsvm"))
            rec = {"name": name, "uri": uri, "read_threads": threads,
                   "sec_per_epoch": round(dt / args.epochs, 4),
                   "rows_per_sec": round(rows / dt, 1),
                   "GBps": round(part * args.epochs / dt / 1e9, 3),
                   "wait_reader_sec_per_epoch": round(
                       (s1["wait_reader_sec"] - s0["wait_reader_sec"]) / args.epochs, 4),
                   "wait_gpu_sec_per_epoch": round(
                       (s1["wait_gpu_sec"] - s0["wait_gpu_sec"]) / args.epochs, 4),
                   "zero_copy": s1.get("zero_copy"), "http": _dmlc.http_stats()}
            out["runs"].append(rec)
            print(json.dumps(rec), file=sys.stderr, flush=True)
        print(json.dumps(out), flush=True)
    finally:
        srv.kill()
        srv.wait()


if __name__ == "__main__":
    main()
