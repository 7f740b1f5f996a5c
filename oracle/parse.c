/* TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's edge-file input (checker and
 * cpu_baseline of bench.py --workload parse; the product path is gs_parse_edges, csrc/parse.hip).
 *
 * ConnectedComponentsExample.getGraphStream (example/ConnectedComponentsExample.java:108-119):
 * every line s of the text file gives
 *     String[] fields = s.split("\\s");
 *     Long src = Long.parseLong(fields[0]), trg = Long.parseLong(fields[1]);
 * so a line is split at every single whitespace character of Java's \s ([ \t\n\x0B\f\r]; two in
 * a row make an empty field, which parseLong rejects), trailing empty fields are dropped by
 * split(), fields past the second are ignored, a field is an optional sign and >= 1 decimal digit
 * within the int64 range, and any other line fails the job. A last line without '\n' counts.
 * Lines are scanned one after another (one host thread). */
#include <stdint.h>

#include "oracle.h"

static int is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\x0B' || c == '\f' || c == '\r'; }

/* Long.parseLong(t[a, b)): 1 on success */
static int parse_long(const char* t, uint64_t a, uint64_t b, int64_t* out) {
    if (a >= b) return 0;
    int neg = 0;
    if (t[a] == '-' || t[a] == '+') { neg = t[a] == '-'; ++a; }
    if (a >= b) return 0;
    const uint64_t lim = neg ? (uint64_t)INT64_MAX + 1 : (uint64_t)INT64_MAX;
    uint64_t v = 0;
    for (uint64_t i = a; i < b; ++i) {
        const char c = t[i];
        if (c < '0' || c > '9') return 0;
        const uint64_t d = (uint64_t)(c - '0');
        if (v > (lim - d) / 10) return 0;
        v = v * 10 + d;
    }
    *out = neg ? (int64_t)(0 - v) : (int64_t)v;
    return 1;
}

int64_t gso_parse_edges(const char* t, uint64_t n, int64_t* src, int64_t* dst, uint64_t cap) {
    uint64_t line = 0, a = 0;
    while (a < n) {
        uint64_t e = a;
        while (e < n && t[e] != '\n') ++e;                 /* [a, e): the line, e = '\n' or end */
        uint64_t b = e;
        while (b > a && is_ws(t[b - 1])) --b;              /* split() drops trailing empty fields */
        uint64_t s1 = a;
        while (s1 < b && !is_ws(t[s1])) ++s1;              /* fields[0] = [a, s1) */
        uint64_t e2 = s1 + 1;                              /* fields[1] starts after ONE separator */
        while (e2 < b && !is_ws(t[e2])) ++e2;
        int64_t x = 0, y = 0;
        if (!(s1 < b && parse_long(t, a, s1, &x) && parse_long(t, s1 + 1, e2, &y))) return -(int64_t)line - 1;
        if (line < cap) { src[line] = x; dst[line] = y; }
        ++line;
        a = e + 1;
    }
    return (int64_t)line;
}
