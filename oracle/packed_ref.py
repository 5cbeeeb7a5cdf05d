"""Independent pure-Python restatement of capnproto-rust's packed codec.

TEST INFRASTRUCTURE ONLY (see oracle/packed_oracle.c): used to cross-check
the C oracle on small inputs.  Written independently of the C restatement
(word-level, bytes objects) so that a slip in one is caught by the other.

    pack(data)                  PackedWrite::write_all  capnp/src/serialize_packed.rs:304-439
    read(data, out_len)         PackedRead::read        capnp/src/serialize_packed.rs:80-228
    read_exact(data, out_len)   io::Read::read_exact    capnp/src/io.rs:16-31
    async_poll_reads(...)       capnp-futures PackedRead::poll_read
                                capnp-futures/src/serialize_packed.rs:87-225
"""

OK = 0
PREMATURE_END_OF_PACKED_INPUT = 2
DID_NOT_END_CLEANLY = 3
FAILED_TO_FILL_WHOLE_BUFFER = 4
MISALIGNED_LEN = 11


def _tag(word: bytes) -> int:
    return sum(1 << k for k, b in enumerate(word) if b)


def pack(data: bytes) -> bytes:
    """PACK one chunk (serialize_packed.rs:304-439)."""
    if len(data) % 8:
        raise ValueError("packed input must be a whole number of words")
    words = [data[i:i + 8] for i in range(0, len(data), 8)]
    out = bytearray()
    i, n = 0, len(words)
    while i < n:
        w = words[i]
        t = _tag(w)
        out.append(t)
        out.extend(b for b in w if b)
        i += 1
        if t == 0x00:                      # zero run (:375-393)
            r = 0
            while r < 255 and i + r < n and words[i + r] == b"\0" * 8:
                r += 1
            out.append(r)
            i += r
        elif t == 0xFF:                    # literal run (:394-433)
            r = 0
            while r < 255 and i + r < n and words[i + r].count(0) < 2:
                r += 1
            out.append(r)
            for j in range(r):
                out.extend(words[i + j])
            i += r
    return bytes(out)


def read(data: bytes, out_len: int):
    """One PackedRead::read over a slice.  Returns (status, out, consumed, nread);
    consumed is where the reference leaves the &[u8] reader: all of it on
    PrematureEnd (refresh_buffer! consumes first, :59-74) and FailedToFill,
    nothing on DidNotEndCleanly."""
    if out_len == 0:
        return OK, b"", 0, 0
    if out_len % 8:
        return MISALIGNED_LEN, b"", 0, 0
    if not data:
        return OK, b"", 0, 0
    out = bytearray()
    ip = 0
    while len(out) < out_len:
        if ip >= len(data):
            return PREMATURE_END_OF_PACKED_INPUT, bytes(out), ip, 0
        t = data[ip]
        ip += 1
        for k in range(8):
            if t >> k & 1:
                if ip >= len(data):
                    return PREMATURE_END_OF_PACKED_INPUT, bytes(out), ip, 0
                out.append(data[ip])
                ip += 1
            else:
                out.append(0)
        if t in (0x00, 0xFF):
            if ip >= len(data):
                return PREMATURE_END_OF_PACKED_INPUT, bytes(out), ip, 0
            run = data[ip] * 8
            ip += 1
            if run > out_len - len(out):
                # returned before any consume (serialize_packed.rs:166-170):
                # a slice reader stays where it was
                return DID_NOT_END_CLEANLY, bytes(out), 0, 0
            if t == 0x00:
                out.extend(b"\0" * run)
            else:
                chunk = data[ip:ip + run]
                out.extend(chunk)
                ip += len(chunk)
                if len(chunk) < run:
                    return FAILED_TO_FILL_WHOLE_BUFFER, bytes(out), ip, 0
    return OK, bytes(out), ip, out_len


def read_exact(data: bytes, out_len: int):
    """read_exact over PackedRead: (status, out, consumed)."""
    st, out, used, nread = read(data, out_len)
    if st == OK and nread != out_len:
        st = FAILED_TO_FILL_WHOLE_BUFFER
    return st, out, used


def async_poll_reads(packed, size, inner_max=1 << 30):
    """capnp-futures PackedRead::poll_read (capnp-futures/src/
    serialize_packed.rs:87-225: stages Start :101-141, WritingZeroes
    :142-155, BufferingWord :156-172, DrainingBuffer :173-198,
    WritingPassthrough :199-221) over a slice reader that returns up to
    `inner_max` bytes a read, polled with reads of `size` bytes until one
    returns 0 bytes or UnexpectedEof.  Returns (the bytes handed out, b"" for
    the clean end or "EOF" for UnexpectedEof)."""
    data, pos = bytes(packed), 0
    st = {"stage": "start", "buf": [0] * 10, "bp": 0, "bs": 10, "bit": 0, "rem": 0}

    def inner(n):
        nonlocal pos
        b = data[pos:pos + min(n, inner_max)]
        pos += len(b)
        return b

    def poll():
        while True:
            s = st["stage"]
            if s == "start":
                b = inner(2 - st["bp"])
                if not b:
                    return "EOF" if st["bp"] > 0 else b""
                st["buf"][st["bp"]:st["bp"] + len(b)] = list(b)
                st["bp"] += len(b)
                if st["bp"] >= 2:
                    tag, cnt = st["buf"][0], st["buf"][1]
                    if tag == 0:
                        st["stage"], st["rem"] = "zero", (cnt + 1) * 8
                    else:
                        st["stage"] = "buffering"
                        st["bs"] = bin(tag).count("1") + 1
                        if st["bs"] == 9:
                            st["bs"] = 10
                        if st["bp"] >= st["bs"]:
                            st["stage"], st["bp"], st["bit"] = "drain", 1, 0
            elif s == "zero":
                k = min(size, st["rem"])
                if k >= st["rem"]:
                    st["bp"], st["stage"] = 0, "start"
                else:
                    st["rem"] -= k
                return bytes(k)
            elif s == "buffering":
                b = inner(st["bs"] - st["bp"])
                if not b:
                    return "EOF"
                st["buf"][st["bp"]:st["bp"] + len(b)] = list(b)
                st["bp"] += len(b)
                if st["bp"] >= st["bs"]:
                    st["stage"], st["bp"], st["bit"] = "drain", 1, 0
            elif s == "drain":
                out = []
                while len(out) < size and st["bit"] < 8:
                    nz = (st["buf"][0] >> st["bit"]) & 1
                    out.append(st["buf"][st["bp"]] if nz else 0)
                    st["bp"] += nz
                    st["bit"] += 1
                if st["bit"] == 8:
                    if st["bp"] == st["bs"]:
                        st["stage"] = "start"
                    else:
                        st["rem"], st["stage"] = st["buf"][st["bp"]] * 8, "pass"
                    st["bp"] = 0
                return bytes(out)
            else:  # pass
                ub = min(st["rem"], size)
                if ub == 0:
                    st["stage"] = "start"
                    continue
                b = inner(ub)
                if not b:
                    return "EOF"
                if len(b) >= st["rem"]:
                    st["stage"] = "start"
                st["rem"] -= len(b)
                return b

    got = b""
    while True:
        r = poll()
        if r == "EOF" or r == b"":
            return got, r
        got += r
