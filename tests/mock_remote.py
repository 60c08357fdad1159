"""In-process mock object stores for the remote filesystem tests (no network):
an S3 endpoint that *verifies* AWS Signature V4 with hashlib/hmac, an Azure
Blob endpoint that verifies SharedKey signatures, and a plain HTTP server
with Range support.  Listing pages are tiny so pagination is exercised."""
from __future__ import annotations

import base64
import hashlib
import hmac
import re
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, Optional


def _range(header: Optional[str], size: int):
    if not header:
        return None
    m = re.match(r"bytes=(\d+)-(\d*)", header)
    b = int(m.group(1))
    e = int(m.group(2)) if m.group(2) else size - 1
    return b, min(e, size - 1)


class _Base(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    server_version = "mock"

    def log_message(self, *a):  # quiet
        pass

    def _send(self, code, body=b"", headers=None):
        self.send_response(code)
        for k, v in (headers or {}).items():
            self.send_header(k, v)
        if "Content-Length" not in (headers or {}):
            self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        if self.command != "HEAD" and body:
            self.wfile.write(body)

    def _body(self) -> bytes:
        n = int(self.headers.get("Content-Length", "0") or 0)
        return self.rfile.read(n) if n else b""

    def _serve_object(self, data: bytes, range_header: Optional[str]):
        r = _range(range_header, len(data))
        if r is None:
            self._send(200, data, {"Content-Length": str(len(data))})
        else:
            b, e = r
            chunk = data[b:e + 1]
            self._send(206, chunk, {"Content-Length": str(len(chunk)),
                                    "Content-Range": f"bytes {b}-{e}/{len(data)}"})


# ----------------------------------------------------------------------------- S3
class S3Handler(_Base):
    store: Dict[str, bytes] = {}
    uploads: Dict[str, Dict[int, bytes]] = {}
    secret = "secret"
    region = "us-east-1"
    page = 2
    requests = 0
    heads = 0

    def _verify(self) -> bool:
        auth = self.headers.get("Authorization")
        if auth is None:
            return False
        m = re.match(r"AWS4-HMAC-SHA256 Credential=([^/]+)/(\d+)/([^/]+)/s3/aws4_request, "
                     r"SignedHeaders=([^,]+), Signature=([0-9a-f]+)", auth)
        if not m:
            return False
        _ak, day, region, names, sig = m.groups()
        u = urllib.parse.urlsplit(self.path)
        q = urllib.parse.parse_qsl(u.query, keep_blank_values=True)
        cq = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(v, safe='-_.~')}"
                      for k, v in sorted(q))
        hdrs = "".join(f"{n}:{self.headers.get(n).strip()}\n" for n in names.split(";"))
        creq = "\n".join([self.command, u.path, cq, hdrs, names,
                          self.headers.get("x-amz-content-sha256")])
        sts = "\n".join(["AWS4-HMAC-SHA256", self.headers.get("x-amz-date"),
                         f"{day}/{region}/s3/aws4_request", hashlib.sha256(creq.encode()).hexdigest()])
        k = hmac.new(("AWS4" + self.secret).encode(), day.encode(), hashlib.sha256).digest()
        for part in (region, "s3", "aws4_request"):
            k = hmac.new(k, part.encode(), hashlib.sha256).digest()
        want = hmac.new(k, sts.encode(), hashlib.sha256).hexdigest()
        return hmac.compare_digest(want, sig)

    def _route(self):
        type(self).requests += 1
        if not self._verify():
            self._send(403, b"<Error><Code>SignatureDoesNotMatch</Code></Error>")
            return None
        u = urllib.parse.urlsplit(self.path)
        parts = urllib.parse.unquote(u.path).lstrip("/").split("/", 1)
        bucket, key = parts[0], parts[1] if len(parts) > 1 else ""
        return bucket, key, dict(urllib.parse.parse_qsl(u.query, keep_blank_values=True))

    def do_HEAD(self):
        type(self).heads += 1
        r = self._route()
        if r is None:
            return
        bucket, key, _ = r
        data = self.store.get(f"{bucket}/{key}")
        if data is None:
            self._send(404)
        else:
            self._send(200, b"", {"Content-Length": str(len(data))})

    def do_GET(self):
        r = self._route()
        if r is None:
            return
        bucket, key, q = r
        if q.get("list-type") == "2":
            self._list(bucket, q)
            return
        data = self.store.get(f"{bucket}/{key}")
        if data is None:
            self._send(404, b"<Error><Code>NoSuchKey</Code></Error>")
        else:
            self._serve_object(data, self.headers.get("Range"))

    def _list(self, bucket, q):
        prefix, delim = q.get("prefix", ""), q.get("delimiter", "")
        maxk = int(q.get("max-keys", "1000"))
        items = []
        for full in sorted(self.store):
            b, k = full.split("/", 1)
            if b != bucket or not k.startswith(prefix):
                continue
            rest = k[len(prefix):]
            if delim and delim in rest:
                p = prefix + rest.split(delim)[0] + delim
                if ("P", p) not in items:
                    items.append(("P", p))
            else:
                items.append(("K", k))
        start = int(q.get("continuation-token", "0") or 0)
        n = min(maxk, self.page)
        page = items[start:start + n]
        trunc = start + n < len(items)
        xml = ["<ListBucketResult>", f"<KeyCount>{len(page)}</KeyCount>",
               f"<IsTruncated>{'true' if trunc else 'false'}</IsTruncated>"]
        if trunc:
            xml.append(f"<NextContinuationToken>{start + n}</NextContinuationToken>")
        for kind, v in page:
            if kind == "K":
                xml.append(f"<Contents><Key>{v}</Key><Size>{len(self.store[bucket + '/' + v])}"
                           "</Size></Contents>")
            else:
                xml.append(f"<CommonPrefixes><Prefix>{v}</Prefix></CommonPrefixes>")
        xml.append("</ListBucketResult>")
        self._send(200, "".join(xml).encode(), {"Content-Type": "application/xml"})

    def do_PUT(self):
        r = self._route()
        if r is None:
            return
        bucket, key, q = r
        body = self._body()
        if "uploadId" in q:
            self.uploads[q["uploadId"]][int(q["partNumber"])] = body
            self._send(200, b"", {"ETag": f'"etag{q["partNumber"]}"'})
        else:
            self.store[f"{bucket}/{key}"] = body
            self._send(200)

    def do_POST(self):
        r = self._route()
        if r is None:
            return
        bucket, key, q = r
        body = self._body()
        if "uploads" in q:
            uid = f"up{len(self.uploads)}"
            self.uploads[uid] = {}
            self._send(200, f"<InitiateMultipartUploadResult><UploadId>{uid}</UploadId>"
                            "</InitiateMultipartUploadResult>".encode())
        elif "uploadId" in q:
            parts = self.uploads.pop(q["uploadId"])
            nums = [int(x) for x in re.findall(rb"<PartNumber>(\d+)</PartNumber>", body)]
            self.store[f"{bucket}/{key}"] = b"".join(parts[i] for i in nums)
            self._send(200, b"<CompleteMultipartUploadResult/>")
        else:
            self._send(400)


# -------------------------------------------------------------------------- Azure
class AzureHandler(_Base):
    store: Dict[str, bytes] = {}
    blocks: Dict[str, bytes] = {}
    account = "acct"
    key = base64.b64encode(b"azure-secret-key").decode()
    page = 2

    def _verify(self) -> bool:
        auth = self.headers.get("Authorization", "")
        m = re.match(r"SharedKey ([^:]+):(.+)", auth)
        if not m:
            return False
        u = urllib.parse.urlsplit(self.path)
        xms = sorted((k.lower(), v.strip()) for k, v in self.headers.items()
                     if k.lower().startswith("x-ms-"))
        canon_h = "".join(f"{k}:{v}\n" for k, v in xms)
        canon_r = f"/{self.account}{u.path}"
        for k, v in sorted(urllib.parse.parse_qsl(u.query, keep_blank_values=True)):
            canon_r += f"\n{k.lower()}:{v}"
        length = self.headers.get("Content-Length", "")
        if length == "0":
            length = ""
        sts = "\n".join([self.command, "", "", length, "", self.headers.get("Content-Type", ""),
                         "", "", "", "", "", ""]) + "\n" + canon_h + canon_r
        want = base64.b64encode(hmac.new(base64.b64decode(self.key), sts.encode(),
                                         hashlib.sha256).digest()).decode()
        return hmac.compare_digest(want, m.group(2))

    def _route(self):
        if not self._verify():
            self._send(403, b"<Error><Code>AuthenticationFailed</Code></Error>")
            return None
        u = urllib.parse.urlsplit(self.path)
        parts = urllib.parse.unquote(u.path).lstrip("/").split("/", 1)
        return parts[0], parts[1] if len(parts) > 1 else "", dict(
            urllib.parse.parse_qsl(u.query, keep_blank_values=True))

    def do_HEAD(self):
        r = self._route()
        if r is None:
            return
        c, b, _ = r
        data = self.store.get(f"{c}/{b}")
        self._send(404) if data is None else self._send(200, b"", {"Content-Length": str(len(data))})

    def do_GET(self):
        r = self._route()
        if r is None:
            return
        c, b, q = r
        if q.get("comp") == "list":
            prefix, delim = q.get("prefix", ""), q.get("delimiter", "")
            items = []
            for full in sorted(self.store):
                cc, k = full.split("/", 1)
                if cc != c or not k.startswith(prefix):
                    continue
                rest = k[len(prefix):]
                if delim and delim in rest:
                    p = prefix + rest.split(delim)[0] + delim
                    if ("P", p) not in items:
                        items.append(("P", p))
                else:
                    items.append(("B", k))
            start = int(q.get("marker", "0") or 0)
            n = min(int(q.get("maxresults", "5000")), self.page)
            page = items[start:start + n]
            xml = ["<EnumerationResults><Blobs>"]
            for kind, v in page:
                if kind == "B":
                    xml.append(f"<Blob><Name>{v}</Name><Properties><Content-Length>"
                               f"{len(self.store[c + '/' + v])}</Content-Length></Properties></Blob>")
                else:
                    xml.append(f"<BlobPrefix><Name>{v}</Name></BlobPrefix>")
            xml.append("</Blobs>")
            xml.append(f"<NextMarker>{start + n if start + n < len(items) else ''}</NextMarker>")
            xml.append("</EnumerationResults>")
            self._send(200, "".join(xml).encode())
            return
        data = self.store.get(f"{c}/{b}")
        if data is None:
            self._send(404)
        else:
            self._serve_object(data, self.headers.get("x-ms-range") or self.headers.get("Range"))

    def do_PUT(self):
        r = self._route()
        if r is None:
            return
        c, b, q = r
        body = self._body()
        if q.get("comp") == "block":
            self.blocks[q["blockid"]] = body
            self._send(201)
        elif q.get("comp") == "blocklist":
            ids = re.findall(rb"<Latest>([^<]+)</Latest>", body)
            self.store[f"{c}/{b}"] = b"".join(self.blocks.pop(i.decode()) for i in ids)
            self._send(201)
        else:
            self.store[f"{c}/{b}"] = body
            self._send(201)


# --------------------------------------------------------------------------- HTTP
class PlainHandler(_Base):
    store: Dict[str, bytes] = {}
    chunked = False  # answer GETs with Transfer-Encoding: chunked bodies
    proxied = 0  # requests that came in proxy form (absolute URL as the target)

    def _key(self):
        if self.path.startswith("http://"):  # a forward-proxy request to this same server
            type(self).proxied += 1
            return urllib.parse.urlsplit(self.path).path
        return self.path

    def do_HEAD(self):
        data = self.store.get(self._key())
        self._send(404) if data is None else self._send(200, b"", {"Content-Length": str(len(data))})

    def do_GET(self):
        data = self.store.get(self._key())
        if data is None:
            self._send(404)
        elif self.chunked:
            b, e = _range(self.headers.get("Range"), len(data)) or (0, len(data) - 1)
            body = data[b:e + 1]
            self.send_response(206)
            self.send_header("Transfer-Encoding", "chunked")
            self.end_headers()
            for i in range(0, len(body), 65536):
                part = body[i:i + 65536]
                self.wfile.write(b"%x\r\n" % len(part) + part + b"\r\n")
            self.wfile.write(b"0\r\n\r\n")
        else:
            self._serve_object(data, self.headers.get("Range"))


# ------------------------------------------------------------------------ WebHDFS
class WebHdfsHandler(_Base):
    """Namenode + datanode in one server: namenode ops OPEN/CREATE/APPEND answer
    307 with a Location under /dn/ (the datanode), as a real cluster does.
    Listings come in pages of 2 via LISTSTATUS_BATCH unless `batch` is off
    (then the op is rejected with 400, as pre-2.8 namenodes do)."""
    store: Dict[str, bytes] = {}
    batch = True
    namenode_bodies = 0  # requests that sent data to the namenode (must stay 0)
    users: set = set()

    def _split(self):
        u = urllib.parse.urlsplit(self.path)
        q = dict(urllib.parse.parse_qsl(u.query))
        return urllib.parse.unquote(u.path), q

    def _json(self, code, obj):
        import json
        self._send(code, json.dumps(obj).encode(), None)

    def _missing(self, p):
        self._json(404, {"RemoteException": {"exception": "FileNotFoundException",
                                             "javaClassName": "java.io.FileNotFoundException",
                                             "message": f"File does not exist: {p}"}})

    def _status(self, p, suffix):
        if p in self.store:
            return {"pathSuffix": suffix, "type": "FILE", "length": len(self.store[p]),
                    "ecPolicyObj": {"name": "RS-6-3", "schema": {"codecName": "rs"}}}
        return {"pathSuffix": suffix, "type": "DIRECTORY", "length": 0}

    def _is_dir(self, p):
        pre = p.rstrip("/") + "/"
        return p == "/" or any(k.startswith(pre) for k in self.store)

    def _children(self, p):
        pre = p.rstrip("/") + "/"
        names = sorted({k[len(pre):].split("/")[0] for k in self.store if k.startswith(pre)})
        return [(n, pre + n) for n in names]

    def _redirect(self, path, q):
        self.users.add(q.get("user.name", ""))
        if int(self.headers.get("Content-Length", "0") or 0):
            type(self).namenode_bodies += 1
            self._body()
        host = self.headers["Host"]
        loc = f"http://{host}/dn{urllib.parse.quote(path)}?" + urllib.parse.urlencode(q)
        self._send(307, b"", {"Location": loc, "Content-Length": "0"})

    def do_GET(self):
        path, q = self._split()
        if path.startswith("/dn/"):
            data = self.store[path[3:]]
            off, n = int(q.get("offset", 0)), int(q.get("length", len(data)))
            return self._send(200, data[off:off + n])
        assert path.startswith("/webhdfs/v1")
        p = path[len("/webhdfs/v1"):] or "/"
        op = q["op"]
        self.users.add(q.get("user.name", ""))
        if op == "GETFILESTATUS":
            if p not in self.store and not self._is_dir(p):
                return self._missing(p)
            return self._json(200, {"FileStatus": self._status(p, "")})
        if op in ("LISTSTATUS", "LISTSTATUS_BATCH"):
            if op == "LISTSTATUS_BATCH" and not self.batch:
                exc = {"exception": "IllegalArgumentException",
                       "message": "Invalid value for webhdfs parameter \"op\""}
                return self._json(400, {"RemoteException": exc})
            if p in self.store:
                kids = [("", p)]
            elif self._is_dir(p):
                kids = self._children(p)
            else:
                return self._missing(p)
            if op == "LISTSTATUS":
                sts = [self._status(f, n) for n, f in kids]
                return self._json(200, {"FileStatuses": {"FileStatus": sts}})
            after = q.get("startAfter")
            if after:
                kids = [k for k in kids if k[0] > after]
            page = kids[:2]
            return self._json(200, {"DirectoryListing": {
                "partialListing": {"FileStatuses": {"FileStatus": [self._status(f, n) for n, f in page]}},
                "remainingEntries": len(kids) - len(page)}})
        if op == "OPEN":
            if p not in self.store:
                return self._missing(p)
            return self._redirect(p, q)
        self._send(400)

    def do_PUT(self):
        path, q = self._split()
        if path.startswith("/dn/"):
            assert q["op"] == "CREATE"
            self.store[path[3:]] = self._body()
            return self._send(201, b"", {"Location": "webhdfs://" + path[3:]})
        self._redirect(path[len("/webhdfs/v1"):], q)

    def do_POST(self):
        path, q = self._split()
        if path.startswith("/dn/"):
            assert q["op"] == "APPEND"
            p = path[3:]
            if p not in self.store:
                return self._missing(p)
            self.store[p] = self.store[p] + self._body()
            return self._send(200)
        self._redirect(path[len("/webhdfs/v1"):], q)


def serve(handler):
    """Start a server on 127.0.0.1:<free port> in a daemon thread."""
    srv = ThreadingHTTPServer(("127.0.0.1", 0), handler)
    srv.daemon_threads = True
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def serve_tls(handler, certfile, keyfile):
    """serve() over TLS (the listening socket wrapped: each accepted
    connection handshakes with the given self-signed certificate)."""
    import ssl
    srv = ThreadingHTTPServer(("127.0.0.1", 0), handler)
    srv.daemon_threads = True
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.load_cert_chain(certfile, keyfile)
    srv.socket = ctx.wrap_socket(srv.socket, server_side=True)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv
