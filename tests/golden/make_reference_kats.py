"""Extract the reference's own known-answer vectors into tests/golden/reference_kats.json.

Run in the build container (needs /root/reference, read-only); the JSON output is
committed and is what the tests read (the GPU box has no /root/reference).

Every vector is taken from the quoted hex literal on a cited line of the reference's
#[cfg(test)] modules (paths relative to /root/reference/anothertls/src). Only data is
extracted — no reference source text is stored.
"""
import json
import os
import re
import sys

REF = "/root/reference/anothertls/src"
QUOTED = re.compile(r'"([^"]*)"')
HEXSTR = re.compile(r"^[0-9A-Fa-f]*$")


def lit(path, line, idx=0):
    with open(os.path.join(REF, path)) as f:
        text = f.readlines()[line - 1]
    found = [q for q in QUOTED.findall(text) if HEXSTR.match(q)]
    return found[idx].lower()


def cite(path, line):
    return f"anothertls/src/{path}:{line}"


def main(out):
    g = "crypto/aes/gcm.rs"
    K = lit(g, 212)
    P4 = lit(g, 213)
    A4 = lit(g, 215)
    gcm = [
        dict(name="gcm_test_decrypt_tc3_roundtrip", key=lit(g, 173), pt=lit(g, 174), iv=lit(g, 175),
             aad=lit(g, 176), tag=lit(g, 179), src=cite(g, 171)),
        dict(name="gcm_tc1", key=lit(g, 188), pt=lit(g, 189), iv=lit(g, 190), aad=lit(g, 191),
             ct="", tag=lit(g, 196), src=cite(g, 186)),
        dict(name="gcm_tc2", key=lit(g, 188), pt=lit(g, 199), iv=lit(g, 190), aad=lit(g, 191),
             tag=lit(g, 202), src=cite(g, 199)),
        dict(name="gcm_tc3", key=lit(g, 205), pt=lit(g, 206), iv=lit(g, 207), aad=lit(g, 191),
             tag=lit(g, 209), src=cite(g, 205)),
        dict(name="gcm_tc4", key=K, pt=P4, iv=lit(g, 214), aad=A4, tag=lit(g, 217), src=cite(g, 212)),
        dict(name="gcm_tc5_iv64", key=K, pt=P4, iv=lit(g, 220), aad=A4, tag=lit(g, 222), src=cite(g, 220)),
        dict(name="gcm_tc6_iv480", key=K, pt=P4, iv=lit(g, 225), aad=A4, tag=lit(g, 227), src=cite(g, 225)),
        dict(name="gcm_tc7_aes192", key=lit(g, 230), pt=lit(g, 232), iv=lit(g, 231), aad=lit(g, 233),
             tag=lit(g, 235), src=cite(g, 230)),
        dict(name="gcm_tc8_aes192", key=lit(g, 230), pt=lit(g, 238), iv=lit(g, 231), aad=lit(g, 233),
             tag=lit(g, 240), src=cite(g, 238)),
    ]
    # AES block KATs (FIPS-197 C.1-C.3), crypto/aes/cipher.rs:420-456: byte arrays, not hex strings.
    a = "crypto/aes/cipher.rs"
    with open(os.path.join(REF, a)) as f:
        lines = f.readlines()

    def arr(start, end):
        s = "".join(lines[start - 1:end])
        body = s[s.index("[", s.index("=")) + 1:s.rindex("]")]
        return "".join("%02x" % int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{2})", body))

    pt = arr(421, 424)
    aes = [
        dict(name="aes128_fips197_c1", key=arr(426, 429), pt=pt, ct=arr(430, 433), src=cite(a, 426)),
        dict(name="aes192_fips197_c2", key=arr(436, 439), pt=pt, ct=arr(440, 443), src=cite(a, 436)),
        dict(name="aes256_fips197_c3", key=arr(446, 450), pt=pt, ct=arr(451, 454), src=cite(a, 446)),
    ]
    c = "crypto/chacha20/cipher.rs"
    chacha = [dict(name="chacha20_rfc8439_2_4_2", key=lit(c, 121), iv=lit(c, 122), counter=1,
                   pt=lit(c, 124), ct=lit(c, 128), src=cite(c, 118))]
    p = "crypto/chacha20/poly1305.rs"
    poly = dict(
        mac=[dict(name="poly1305_rfc8439_2_5_2", key=lit(p, 115), msg=lit(p, 117), tag=lit(p, 119),
                  src=cite(p, 112))],
        key_gen=[dict(name="poly1305_keygen_rfc8439_2_6_2", key=lit(p, 127), iv=lit(p, 128),
                      otk=lit(p, 130), src=cite(p, 124))],
        aead=[
            dict(name="chacha_poly_rfc8439_2_8_2", pt=lit(p, 136), aad=lit(p, 137), key=lit(p, 139),
                 iv=lit(p, 140), ct=lit(p, 141), tag=lit(p, 142), src=cite(p, 134)),
            dict(name="chacha_poly_rfc8439_a5_decrypt", ct=lit(p, 160), key=lit(p, 163), aad=lit(p, 164),
                 tag=lit(p, 165), iv=lit(p, 166), pt=lit(p, 167), src=cite(p, 158)),
        ],
    )
    s2, s3 = "hash/sha256.rs", "hash/sha384.rs"
    fox, cog = "The quick brown fox jumps over the lazy dog", "The quick brown fox jumps over the lazy cog"
    sha = [
        dict(hash="sha256", msg="", digest=lit(s2, 212), src=cite(s2, 212)),
        dict(hash="sha256", msg=fox.encode().hex(), digest=lit(s2, 216), src=cite(s2, 216)),
        dict(hash="sha256", msg=cog.encode().hex(), digest=lit(s2, 220), src=cite(s2, 220)),
        dict(hash="sha384", msg="", digest=lit(s3, 230, -1), src=cite(s3, 230)),
        dict(hash="sha384", msg=fox.encode().hex(), digest=lit(s3, 231, -1), src=cite(s3, 231)),
        dict(hash="sha384", msg=cog.encode().hex(), digest=lit(s3, 232, -1), src=cite(s3, 232)),
    ]
    hm = "hash/hmac.rs"
    hmac = [
        dict(hash="sha256", key=lit(hm, 103), data=lit(hm, 104), mac=lit(hm, 106), src=cite(hm, 106)),
        dict(hash="sha384", key=lit(hm, 103), data=lit(hm, 104), mac=lit(hm, 107), src=cite(hm, 107)),
        dict(hash="sha256", key=lit(hm, 111), data=lit(hm, 112), mac=lit(hm, 114), src=cite(hm, 114)),
        dict(hash="sha384", key=lit(hm, 111), data=lit(hm, 112), mac=lit(hm, 115), src=cite(hm, 115)),
    ]
    hk = "hash/hkdf.rs"
    hkdf = [
        dict(hash="sha256", ikm=lit(hk, 87), salt=lit(hk, 88), info=lit(hk, 89), okm=lit(hk, 90), src=cite(hk, 86)),
        dict(hash="sha256", ikm=lit(hk, 94), salt=lit(hk, 95), info=lit(hk, 96), okm=lit(hk, 97), src=cite(hk, 93)),
        dict(hash="sha256", ikm=lit(hk, 101), salt=lit(hk, 102), info=lit(hk, 103), okm=lit(hk, 104), src=cite(hk, 100)),
    ]
    doc = dict(
        about="Known-answer vectors from otsmr/AnotherTLS v0.1.3 unit tests (see 'src' per vector). "
              "Generated by tests/golden/make_reference_kats.py.",
        aes_block=aes, gcm=gcm, chacha20=chacha, poly1305=poly, sha=sha, hmac=hmac, hkdf=hkdf,
    )
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "reference_kats.json"))
