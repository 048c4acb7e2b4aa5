"""Pure-Python twin of the reference CPU path -- TEST INFRASTRUCTURE ONLY.

Restates, line for line in behaviour, the Freebirdgo/MapReduce_Rust worker data path:

  wc::map            src/app/wc.rs:6-13     delete [^\\w\\s] (Unicode), split_whitespace, emit (tok, "1")
  wc::reduce         src/app/wc.rs:15-17    values.len().to_string()
  cal_hash_for_key   src/mr/worker.rs:111-115  std DefaultHasher = SipHash-1-3, keys (0,0), bytes ++ 0xFF
  write_key_value_to_file  worker.rs:117-140  "k v\\n" appended to mr-{m}-{h % R}.txt in token order
  read_file_to_mem_reduce  worker.rs:79-109   concat mr-{m}-{r}.txt for m in 0..map_n, split "\\n"/" "
  Worker::reduce     worker.rs:157-193      stable sort by key bytes, group adjacent, LAST GROUP NEVER WRITTEN
  generate_output    src/run.sh:16-20       cat mr-* | sort  (LC_ALL=C) > final.txt

The reference cannot be built here (Rust toolchain absent), so this twin and the C
restatement in oracle/ are cross-checked against each other and against the golden digests recorded
in SURVEY.md §8(c).  Used only to generate fixtures in this container and by CPU tests.
"""
import regex

_DELETE = regex.compile(r"[^\w\s]")   # wc.rs:7
_TOKEN = regex.compile(r"\S+")          # split_whitespace: maximal non-White_Space runs


def wc_map(text):
    """wc.rs:6-13 -> list of (key, "1") in input order."""
    return [(t, "1") for t in _TOKEN.findall(_DELETE.sub("", text))]


def wc_reduce(key, values):
    """wc.rs:15-17."""
    return str(len(values))


def tokens(text):
    return [k for k, _ in wc_map(text)]


_M64 = (1 << 64) - 1


def _rotl(x, b):
    return ((x << b) | (x >> (64 - b))) & _M64


def siphash(data, c_rounds=1, d_rounds=3, k0=0, k1=0):
    """SipHash-c-d over `data` (bytes).  Rust DefaultHasher = SipHash-1-3 with k0 = k1 = 0."""
    v0 = k0 ^ 0x736F6D6570736575
    v1 = k1 ^ 0x646F72616E646F6D
    v2 = k0 ^ 0x6C7967656E657261
    v3 = k1 ^ 0x7465646279746573

    def rnd(v0, v1, v2, v3):
        v0 = (v0 + v1) & _M64; v1 = _rotl(v1, 13); v1 ^= v0; v0 = _rotl(v0, 32)
        v2 = (v2 + v3) & _M64; v3 = _rotl(v3, 16); v3 ^= v2
        v0 = (v0 + v3) & _M64; v3 = _rotl(v3, 21); v3 ^= v0
        v2 = (v2 + v1) & _M64; v1 = _rotl(v1, 17); v1 ^= v2; v2 = _rotl(v2, 32)
        return v0, v1, v2, v3

    n = len(data)
    full = n - (n % 8)
    for i in range(0, full, 8):
        m = int.from_bytes(data[i:i + 8], "little")
        v3 ^= m
        for _ in range(c_rounds):
            v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
        v0 ^= m
    b = ((n & 0xFF) << 56) | int.from_bytes(data[full:], "little")
    v3 ^= b
    for _ in range(c_rounds):
        v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
    v0 ^= b
    v2 ^= 0xFF
    for _ in range(d_rounds):
        v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
    return v0 ^ v1 ^ v2 ^ v3


def key_hash(key):
    """worker.rs:111-115: <str as Hash>::hash writes the UTF-8 bytes then 0xFF."""
    return siphash(key.encode("utf-8") + b"\xff")


def partition(key, n_reduce):
    """worker.rs:129: (hash % reduce_n as u64) as i32."""
    return key_hash(key) % n_reduce


def map_task(text, n_reduce):
    """worker.rs:142-155 + 117-140: bytes of mr-{m}-{r}.txt for r in 0..R."""
    parts = [[] for _ in range(n_reduce)]
    for k, v in wc_map(text):
        parts[partition(k, n_reduce)].append(f"{k} {v}\n")
    return ["".join(p).encode("utf-8") for p in parts]


def reduce_task(intermediates, reduce_fn=wc_reduce):
    """worker.rs:157-193 over the list of mr-{m}-{r}.txt contents (m order).  Returns mr-{r}.txt bytes."""
    kvs = []
    for content in intermediates:                         # :84-107
        for line in content.decode("utf-8").split("\n"):
            if not line:
                continue
            f = line.split(" ")
            assert len(f) == 2                            # :100
            kvs.append((f[0], f[1]))
    kvs.sort(key=lambda kv: kv[0].encode("utf-8"))       # :162-164 stable, byte order
    out = []
    vals = []
    prev = ""
    for k, v in kvs:                                      # :169-184
        if not prev:
            prev = k
        if k != prev:
            out.append(f"{prev} {reduce_fn(prev, vals)}\n")
            vals = []
            prev = k
        vals.append(v)
    # the last group is never written (reference behaviour)
    return "".join(out).encode("utf-8")


def wc_job(texts, n_reduce):
    """Whole reference job: map every file, then reduce every partition."""
    inter = [map_task(t, n_reduce) for t in texts]
    outs = [reduce_task([inter[m][r] for m in range(len(texts))]) for r in range(n_reduce)]
    return inter, outs


def final_txt(outs):
    """run.sh:16-20 with LC_ALL=C: concatenate and sort lines bytewise."""
    lines = []
    for o in outs:
        lines.extend(l for l in o.split(b"\n") if l)
    lines.sort()
    return b"".join(l + b"\n" for l in lines)


# ---- indexer (build-defined; there is no indexer in the reference) ----

def indexer_map(text, doc):
    """Emit (word, doc) once per distinct word of the document, first-occurrence order."""
    seen = set()
    out = []
    for t in tokens(text):
        if t not in seen:
            seen.add(t)
            out.append((t, doc))
    return out


def indexer_reduce(key, values):
    vs = sorted(values, key=lambda s: s.encode("utf-8"))
    return f"{len(vs)} {','.join(vs)}"


def indexer_job(texts, docs, n_reduce):
    inter = []
    for text, doc in zip(texts, docs):
        parts = [[] for _ in range(n_reduce)]
        for k, v in indexer_map(text, doc):
            parts[partition(k, n_reduce)].append(f"{k} {v}\n")
        inter.append(["".join(p).encode("utf-8") for p in parts])
    outs = [reduce_task([inter[m][r] for m in range(len(texts))], indexer_reduce) for r in range(n_reduce)]
    return outs
