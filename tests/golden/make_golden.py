"""Writes tests/golden/golden_packing.json: the known-answer vectors that the
reference's own tests hold for the packed codec, as data.

Sources (capnproto-rust checkout, read as text):
  * capnp/src/serialize_packed.rs:506-566   simple_packing (14 unpacked<->packed pairs)
  * capnp/src/serialize_packed.rs:468-475   premature_eof
  * capnp/src/serialize_packed.rs:596-611   did_not_end_cleanly_on_a_segment_boundary
  * capnp/src/serialize_packed.rs:613-634   premature_end_of_packed_input
  * capnp/src/serialize_packed.rs:636-651   packed_segment_table
  * capnp-futures/src/serialize_packed.rs:611-671  simple_packing (async twin: same pairs)
  * capnp-futures/src/serialize_packed.rs:747-761  unpacks_across_partial_output_buffers
  * capnp/src/serialize.rs:742-831          test_read_segment_table
  * capnp/src/serialize.rs:904-935          test_read_invalid_segment_table / overflow
  * capnp/src/serialize.rs:937-1028         test_write_segment_table
The reference is never imported or executed (it is Rust); the vectors below
were transcribed from those test sources.  Re-run this script to regenerate
the JSON; the test suite checks the committed JSON against it.
"""
import json
import os

Z8 = [0] * 8


def packing_pairs():
    p = []
    p.append(([], []))
    p.append((Z8, [0, 0]))
    p.append(([0, 0, 12, 0, 0, 34, 0, 0], [0x24, 12, 34]))
    p.append(([1, 3, 2, 4, 5, 7, 6, 8], [0xff, 1, 3, 2, 4, 5, 7, 6, 8, 0]))
    p.append((Z8 + [1, 3, 2, 4, 5, 7, 6, 8], [0, 0, 0xff, 1, 3, 2, 4, 5, 7, 6, 8, 0]))
    p.append(([0, 0, 12, 0, 0, 34, 0, 0, 1, 3, 2, 4, 5, 7, 6, 8],
              [0x24, 12, 34, 0xff, 1, 3, 2, 4, 5, 7, 6, 8, 0]))
    p.append(([1, 3, 2, 4, 5, 7, 6, 8, 8, 6, 7, 4, 5, 2, 3, 1],
              [0xff, 1, 3, 2, 4, 5, 7, 6, 8, 1, 8, 6, 7, 4, 5, 2, 3, 1]))
    s = [1, 2, 3, 4, 5, 6, 7, 8]
    p.append((s * 4 + [0, 2, 4, 0, 9, 0, 5, 1],
              [0xff] + s + [3] + s * 3 + [0xd6, 2, 4, 9, 5, 1]))
    p.append((s * 2 + [6, 2, 4, 3, 9, 0, 5, 1] + s + [0, 2, 4, 0, 9, 0, 5, 1],
              [0xff] + s + [3] + s + [6, 2, 4, 3, 9, 0, 5, 1] + s + [0xd6, 2, 4, 9, 5, 1]))
    p.append(([8, 0, 100, 6, 0, 1, 1, 2] + Z8 * 3 + [0, 0, 1, 0, 2, 0, 3, 1],
              [0xed, 8, 100, 6, 1, 1, 2, 0, 2, 0xd4, 1, 2, 3, 1]))
    p.append((Z8, [0, 0]))
    p.append((Z8 * 2, [0, 1]))
    p.append((Z8 * 3, [0, 2]))
    p.append((Z8 * 258, [0, 255, 0, 1]))
    return p


def main():
    doc = {
        "source": "capnproto-rust 0.27.0 test vectors, transcribed as data (see make_golden.py)",
        "packing": [
            {"unpacked": u, "packed": k, "ref": "capnp/src/serialize_packed.rs:506-566"}
            for u, k in packing_pairs()
        ],
        # (packed input, output length, expected status name)
        "unpack_errors": [
            {"packed": [], "out_len": 8, "status": "FAILED_TO_FILL_WHOLE_BUFFER",
             "ref": "capnp/src/serialize_packed.rs:468-475 (read_exact on empty input is_err)"},
            {"packed": [0xff, 1, 2, 3, 4, 5, 6, 7, 8, 37, 1, 2], "out_len": 200,
             "status": "DID_NOT_END_CLEANLY", "ref": "capnp/src/serialize_packed.rs:596-611"},
            {"packed": [0xf0, 1, 2], "out_len": 200, "status": "PREMATURE_END_OF_PACKED_INPUT",
             "ref": "capnp/src/serialize_packed.rs:627"},
            {"packed": [0], "out_len": 200, "status": "PREMATURE_END_OF_PACKED_INPUT",
             "ref": "capnp/src/serialize_packed.rs:628"},
            {"packed": [0xff, 1, 2, 3, 4, 5, 6, 7, 8], "out_len": 200,
             "status": "PREMATURE_END_OF_PACKED_INPUT", "ref": "capnp/src/serialize_packed.rs:629"},
            {"packed": [1, 1], "out_len": 200, "status": "PREMATURE_END_OF_PACKED_INPUT",
             "ref": "capnp/src/serialize_packed.rs:633"},
        ],
        "unpacks_to": [
            {"packed": [0x11, 4, 1, 0, 1, 0, 0],
             "unpacked": [4, 0, 0, 0, 1, 0, 0, 0] + [0] * 24,
             "ref": "capnp/src/serialize_packed.rs:636-651"},
            {"packed": [0x81, 42, 99], "unpacked": [42, 0, 0, 0, 0, 0, 0, 99],
             "ref": "capnp-futures/src/serialize_packed.rs:753"},
            {"packed": [0xff, 1, 3, 2, 4, 5, 7, 6, 8, 1, 8, 6, 7, 4, 5, 2, 3, 1],
             "unpacked": [1, 3, 2, 4, 5, 7, 6, 8, 8, 6, 7, 4, 5, 2, 3, 1],
             "ref": "capnp-futures/src/serialize_packed.rs:756-760"},
        ],
        # packed message streams read through serialize_packed::read_message
        "read_message": [
            {"packed": [0x11, 4, 1, 0, 1, 0, 0], "status": "OK", "seg_words": [1, 0, 0, 0, 0],
             "ref": "capnp/src/serialize_packed.rs:650 (5-segment table read in one unit)"},
            {"packed": [], "status": "PREMATURE_END_OF_FILE", "try_status": "NONE",
             "ref": "capnp/src/serialize.rs:796-800 (try_read_empty); serialize.rs:295-297"},
        ],
        # unpacked segment-table words -> segment lengths (serialize.rs:742-831)
        "segment_tables": [
            {"table": [0, 0, 0, 0, 0, 0, 0, 0], "seg_words": [0]},
            {"table": [0, 0, 0, 0, 1, 0, 0, 0], "seg_words": [1]},
            {"table": [1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0], "seg_words": [1, 1]},
            {"table": [2, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0], "seg_words": [1, 1, 256]},
            {"table": [3, 0, 0, 0, 77, 0, 0, 0, 23, 0, 0, 0, 1, 0, 0, 0, 99, 0, 0, 0, 0, 0, 0, 0],
             "seg_words": [77, 23, 1, 99]},
        ],
        # unpacked tables that must be rejected (serialize.rs:904-935)
        "invalid_segment_tables": [
            {"table": [0, 2, 0, 0] + [0] * (513 * 4), "status": "INVALID_NUMBER_OF_SEGMENTS"},
            {"table": [0, 0, 0, 0], "status": "ANY_ERROR"},
            {"table": [0, 0, 0, 0, 0, 0, 0], "status": "ANY_ERROR"},
            {"table": [255, 255, 255, 255], "status": "ANY_ERROR"},
            {"table": [1, 0, 0, 0, 0xff, 0xff, 0xff, 0xff, 2, 0, 0, 0, 0, 0, 0, 0],
             "status": "ANY_ERROR"},
        ],
        # segment lengths -> written (unpacked) table bytes (serialize.rs:937-1028)
        "write_segment_tables": [
            {"seg_words": [0], "table": [0, 0, 0, 0, 0, 0, 0, 0]},
            {"seg_words": [1], "table": [0, 0, 0, 0, 1, 0, 0, 0]},
            {"seg_words": [199], "table": [0, 0, 0, 0, 199, 0, 0, 0]},
            {"seg_words": [0, 1], "table": [1, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0]},
            {"seg_words": [199, 1, 199, 0],
             "table": [3, 0, 0, 0, 199, 0, 0, 0, 1, 0, 0, 0, 199, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0]},
            {"seg_words": [199, 1, 199, 0, 1],
             "table": [4, 0, 0, 0, 199, 0, 0, 0, 1, 0, 0, 0, 199, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0]},
        ],
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_packing.json")
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    return path


if __name__ == "__main__":
    print(main())
