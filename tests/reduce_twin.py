"""Line-by-line Python restatement of the reference's reduce task (TEST INFRASTRUCTURE ONLY).

read_file_to_mem_reduce (src/mr/worker.rs:79-109) + Worker::reduce (worker.rs:157-193) over the
contents of intermediate files mr-{m}-{r}.txt, with wc::reduce (src/app/wc.rs:15-17) = number of values.
The loop keeps the reference's two quirks: `if prev.is_empty() { prev = kv.key }` (:170-172: empty keys
fold into the next group) and no flush after the loop (the last group is dropped) unless drop_last=False.
"""


def ref_reduce(files, drop_last=True):
    kvs = []
    for c in files:
        for line in c.decode("utf-8").split("\n"):
            if not line:
                continue
            f = line.split(" ")
            assert len(f) == 2
            kvs.append((f[0], f[1]))
    kvs.sort(key=lambda kv: kv[0].encode())
    out, prev, vals = [], "", []
    for k, v in kvs:
        if prev == "":
            prev = k
        if k != prev:
            out.append(f"{prev} {len(vals)}\n")
            vals = []
            prev = k
        vals.append(v)
    if not drop_last and vals:
        out.append(f"{prev} {len(vals)}\n")
    return "".join(out).encode()


# intermediate-file edge cases shared by the oracle test and the GPU parity test
REDUCE_EDGE_CASES = [
    [b"b 1\na 1\n", b"a 1\nc 7\n\n\nb x\n"],          # values other than "1" still count 1 each
    [b" 1\n 1\nzz 1\nab 1\n"],                        # empty keys join the first group (prev == "")
    [b" 1\n"],                                        # only empty keys
    [b" 1\n", b" 1\nq 1\n", b"r 1\n"],                # empty keys over several files
    [b"a-b 1\nx\xc3\xa9y 1\na-b 1\nq 1"],             # non-\w key bytes kept verbatim, no final newline
    [("k" * 40 + " 1\n").encode() * 3 + ("k" * 39 + "j 1\n").encode() + b"z 1\n"],  # long keys
    [b"", b"\n\n", b"w 1\n"],                         # empty files and empty lines
    [],
]
