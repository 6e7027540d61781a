"""config.json surface of the reference (MCPT/config.cpp:70-124, MCPT/config.json).

The reference reads ``config.json`` from the working directory with a patched
nlohmann/json 3.1.2 in which ``#`` starts a comment wherever the scanner skips
whitespace (MCPT/json.hpp:3037-3043); ``configid`` selects one entry of the
``config`` array.  :class:`Config` exposes the same getters
(MCPT/config.cpp:128-145, MCPT/config.h:8-30) with the same defaults.
"""
import json


def strip_hash_comments(text):
    """Drop ``# ...`` to end of line outside JSON strings (json.hpp:3037-3043)."""
    out, i, n, in_str = [], 0, len(text), False
    while i < n:
        c = text[i]
        if in_str:
            out.append(c)
            if c == "\\" and i + 1 < n:
                out.append(text[i + 1])
                i += 1
            elif c == '"':
                in_str = False
        elif c == '"':
            in_str = True
            out.append(c)
        elif c == "#":
            while i < n and text[i] != "\n":
                i += 1
            continue
        else:
            out.append(c)
        i += 1
    return "".join(out)


def loads(text):
    return json.loads(strip_hash_comments(text))


class Config:
    """One selected entry of a reference config.json (config.cpp:72-122)."""

    def __init__(self, obj, configid=None):
        if isinstance(obj, str):
            with open(obj, "r") as fh:
                obj = loads(fh.read())
        self.root = obj
        cid = int(obj["configid"] if configid is None else configid)
        c = obj["config"][cid]
        self.entry = c
        self.bvhtype = c.get("bvhtype", "") or "hlbvh"
        self.testall = bool(c.get("testall", False))
        self.directory = c.get("directory", "")
        if self.testall:
            self.objs = c["objname"]
            self.objname = ""
            self.camera = None
            self.width = self.height = 0
            self.testbvh = False
            self.maxdepth = self.attempt = 0
            self.opencl = False
            return
        self.camera = c.get("camera")
        self.objname = c["objname"]
        self.width = int(float(c["width"]))      # read as double, stored as int
        self.height = int(float(c["height"]))
        self.testbvh = bool(c.get("testbvh", False))
        self.objs = None
        if self.testbvh:
            self.maxdepth = self.attempt = 0
            self.opencl = False
            return
        self.platform = c.get("platform", "")
        self.raygenerator = c.get("raygenerator", "")
        self.intersect = c.get("intersect", "")
        self.shade = c.get("shade", "")
        self.opencl = bool(c.get("opencl", False))
        self.maxdepth = int(c["maxdepth"])
        self.attempt = int(c["attempt"])

    # the reference's free-function getters (config.h)
    def WIDTH(self): return self.width
    def HEIGHT(self): return self.height
    def MAXDEPTH(self): return self.maxdepth
    def MAXATTEPMT(self): return self.attempt  # sic, config.h:24
    def GETOBJNAME(self): return self.objname
    def GETDIRECTORY(self): return self.directory
    def GETCAMERA(self): return self.camera
    def BVHTYPE(self): return self.bvhtype
    def TESTBVH(self): return self.testbvh
    def TESTALL(self): return self.testall
    def USEOPENCL(self): return self.opencl
    def GETOBJS(self): return self.objs
