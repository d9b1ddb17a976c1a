#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY — lists the reference's own libcrypto + libssl
source files for an x86-64 Linux/glibc host, by evaluating LibreSSL 2.4.1's
automake lists where they lie:

  src/libressl-2.4.1/crypto/Makefile.am   (+ Makefile.am.elf-x86_64,
                                            Makefile.am.arc4random)
  src/libressl-2.4.1/ssl/Makefile.am

with the conditionals configure would set here (HOST_ASM_ELF_X86_64, HOST_LINUX,
and HAVE_* for what glibc 2.35 provides).  oracle/Makefile compiles the listed
files from /root/reference into oracle/_ref/libssl_ref.so — the reference
record layer (tls1_enc, ssl3_get_record, do_ssl3_write) and its handshake, so
that an unmodified LibreSSL libssl can run with libtlsgpu.so interposed
(BASELINE configs[0]).  Nothing is copied.

usage: ref_sources.py REF_ROOT {crypto|ssl|cflags}
"""
import os
import re
import sys

# configure results for this host (glibc 2.35: no strlcpy/strlcat, no
# arc4random, no timingsafe_*; everything else present)
TRUE = {
    "HOST_ASM_ELF_X86_64", "HOST_LINUX", "OPENSSLDIR_DEFINED",
    "HAVE_EXPLICIT_BZERO", "HAVE_STRNDUP", "HAVE_STRNLEN", "HAVE_ASPRINTF",
    "HAVE_INET_PTON", "HAVE_TIMEGM", "HAVE_REALLOCARRAY", "HAVE_GETENTROPY",
    "HAVE_STRCASECMP", "HAVE_STRSEP", "HAVE_MEMMEM",
}
CFLAG_HAVES = sorted(h for h in TRUE if h.startswith("HAVE_"))


def evaluate(path, var_re, out, cond_stack=None):
    """Collect `<var> += x` / `<var> = x` values of an automake file under the
    conditionals above (if/else/endif, `!` negation, `include`)."""
    base = os.path.dirname(path)
    stack = [] if cond_stack is None else cond_stack
    with open(path) as f:
        for raw in f:
            line = raw.strip()
            m = re.match(r"^if\s+(!?)(\w+)$", line)
            if m:
                val = m.group(2) in TRUE
                stack.append(val if not m.group(1) else not val)
                continue
            if line == "else":
                stack[-1] = not stack[-1]
                continue
            if line == "endif":
                stack.pop()
                continue
            if not all(stack):
                continue
            m = re.match(r"^include\s+(\S+)$", line)
            if m and "top_srcdir" not in m.group(1):
                evaluate(os.path.join(base, m.group(1)), var_re, out, stack)
                continue
            m = re.match(r"^(\w+)\s*\+?=\s*(.*)$", line)
            if m and re.fullmatch(var_re, m.group(1)):
                for tok in m.group(2).split():
                    if tok == "$(ASM_X86_64_ELF)":
                        out.extend(asm_list(base))
                    elif not tok.startswith("$("):
                        out.append(tok)
    return out


def asm_list(crypto_dir):
    out = []
    with open(os.path.join(crypto_dir, "Makefile.am.elf-x86_64")) as f:
        for line in f:
            m = re.match(r"^ASM_X86_64_ELF\s*\+?=\s*(\S+)", line.strip())
            if m:
                out.append(m.group(1))
    return out


def asm_defines(crypto_dir):
    out = []
    with open(os.path.join(crypto_dir, "Makefile.am.elf-x86_64")) as f:
        for line in f:
            m = re.match(r"^libcrypto_la_CPPFLAGS\s*\+=\s*(-D\w+)", line.strip())
            if m:
                out.append(m.group(1))
    return out


def main():
    ref, what = sys.argv[1], sys.argv[2]
    crypto = os.path.join(ref, "crypto")
    if what == "crypto":
        srcs = evaluate(os.path.join(crypto, "Makefile.am"),
                        r"libcrypto_la_SOURCES|libcompat_la_SOURCES", [])
        print(" ".join(s for s in srcs if s.endswith((".c", ".s", ".S"))))
    elif what == "ssl":
        srcs = evaluate(os.path.join(ref, "ssl", "Makefile.am"), r"libssl_la_SOURCES", [])
        print(" ".join(s for s in srcs if s.endswith(".c")))
    elif what == "cflags":
        print(" ".join(asm_defines(crypto) + ["-D" + h for h in CFLAG_HAVES]))
    else:
        raise SystemExit(f"unknown list {what}")


if __name__ == "__main__":
    main()
