/*
 * ingest_oracle.c -- CPU restatement of GeoFlink's point deserializers.
 *
 * TEST INFRASTRUCTURE ONLY (same rule as geohip_oracle.c): loaded by tests/ and bench.py's
 * cpu_baseline leg as the checker / the timed CPU baseline; libgeohip.so never links it.
 *
 * Written independently of the device parser (spatialflink_amd/csrc/ingest_parse.h): the
 * record is first rewritten the way the Java code does it (quote removal, a restated regex
 * split, String.trim), and the numeric token is validated against the Java / JSON grammar and
 * then converted by glibc strtod, which is correctly rounded (ties to even) like
 * Double.parseDouble.  Reference (paths relative to /root/reference/src/main/java/GeoFlink):
 *
 *   CSVTSVToSpatial.map   spatialStreams/Deserialization.java:248-254
 *   CSVTSVToTSpatial.map  spatialStreams/Deserialization.java:306-321 (Long.valueOf timestamp)
 *   GeoJSONToSpatial.map  spatialStreams/Deserialization.java:132-146, readGeoJSON :1554
 *   WKTToSpatial.map      spatialStreams/Deserialization.java:223-228, getCoordinate :1510-1514
 *   Point(x, y, uGrid)    spatialObjects/Point.java:60-66 -> HelperClass.assignGridCellID :104-116
 *
 * Third-party pieces restated from their published behaviour (not vendored in the reference):
 * java.lang.String.split (Java 8: a positive-width match at index 0 yields a leading "",
 * trailing "" are removed), FloatingDecimal.readJavaFormatString (trim, NaN/Infinity, hex,
 * [fFdD] suffix), Long.valueOf, Jackson number grammar + IntNode/LongNode/DoubleNode
 * re-serialisation (jackson-databind via flink-connector-kafka), JTS 1.16.1 GeoJsonReader /
 * WKTReader (StreamTokenizer word characters a-z A-Z 0-9 - + . 160-255, whitespace 0-32).
 * Parity: no reference fixtures exist for the deserializers ("parity unpinned" in DESIGN.md);
 * the known answers in tests/test_ingest.py are derived from the Java grammar by hand.
 *
 * Records are the '\n'-separated lines of a text batch; a final empty line (text ending in
 * '\n') is not a record.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define ING_OK 0
#define ING_ERR -1 /* the reference throws (NumberFormatException, IndexOutOfBounds, ParseException) */
#define ING_UNDECIDED -2 /* valid for the reference, but a form libgeohip does not restate (it hands
                            such records back to the host): the batch is rejected all the same */

enum { FMT_CSV = 0, FMT_GEOJSON = 1, FMT_WKT = 2 };

typedef struct {
    int32_t format, delim, fx, fy, fts, foid; /* foid: csvTsvSchemaAttr.get(0) (trajectory batches) */
} ing_spec;

/* TrajectoryStream's GeoJSON parameters (include/geohip.h geohip_traj_spec) */
typedef struct {
    int32_t date_format, utc_offset_min;
    char prop_ts[60], prop_oid[60];
} ing_traj;

/* a record's objID: bytes [a, b) of buf (the quote-free record copy or the record), or null */
typedef struct {
    int null;
    const char* buf;
    size_t a, b;
} ing_oid;

typedef struct {
    double min_x, min_y, cell_len;
    int32_t n;
} ing_grid;

static int jspace(unsigned char c) { /* java.util.regex \s */
    return c == ' ' || c == '\t' || c == '\n' || c == 0x0b || c == '\f' || c == '\r';
}
static int isdig(unsigned char c) { return c >= '0' && c <= '9'; }
static int ishex(unsigned char c) { return isdig(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }

/* Double.parseDouble(String): FloatingDecimal.readJavaFormatString.  s[0..n) untrimmed. */
static int j_parse_double(const char* s, size_t n, double* out) {
    size_t a = 0, b = n;
    while (a < b && (unsigned char)s[a] <= ' ') a++; /* String.trim */
    while (b > a && (unsigned char)s[b - 1] <= ' ') b--;
    if (a == b) return ING_ERR;
    char buf[512];
    size_t i = a;
    int neg = 0;
    if (s[i] == '+' || s[i] == '-') {
        neg = s[i] == '-';
        i++;
    }
    if (i < b && (s[i] == 'N' || s[i] == 'I')) {
        const char* w = s[i] == 'N' ? "NaN" : "Infinity";
        size_t L = strlen(w);
        if (b - i != L || memcmp(s + i, w, L) != 0) return ING_ERR;
        *out = s[i] == 'N' ? NAN : (neg ? -INFINITY : INFINITY);
        return ING_OK;
    }
    if (i + 1 < b && s[i] == '0' && (s[i + 1] == 'x' || s[i + 1] == 'X')) {
        /* [+-]0[xX] hex* [. hex*] [pP][+-]?digits+ [fFdD]?, at least one hex digit */
        size_t j = i + 2, nh = 0;
        while (j < b && ishex(s[j])) j++, nh++;
        if (j < b && s[j] == '.') {
            j++;
            while (j < b && ishex(s[j])) j++, nh++;
        }
        if (nh == 0 || j >= b || (s[j] != 'p' && s[j] != 'P')) return ING_ERR;
        j++;
        if (j < b && (s[j] == '+' || s[j] == '-')) j++;
        size_t ne = 0;
        while (j < b && isdig(s[j])) j++, ne++;
        if (ne == 0) return ING_ERR;
        size_t end = j;
        if (j < b && strchr("fFdD", s[j])) j++;
        if (j != b || end - a >= sizeof buf) return ING_ERR;
        memcpy(buf, s + a, end - a);
        buf[end - a] = 0;
        *out = strtod(buf, NULL); /* C99 hex conversion, correctly rounded */
        return ING_OK;
    }
    size_t j = i, nd = 0;
    while (j < b && isdig(s[j])) j++, nd++;
    if (j < b && s[j] == '.') {
        j++;
        while (j < b && isdig(s[j])) j++, nd++;
    }
    if (nd == 0) return ING_ERR;
    if (j < b && (s[j] == 'e' || s[j] == 'E')) {
        j++;
        if (j < b && (s[j] == '+' || s[j] == '-')) j++;
        size_t ne = 0;
        while (j < b && isdig(s[j])) j++, ne++;
        if (ne == 0) return ING_ERR;
    }
    size_t end = j;
    if (j < b && strchr("fFdD", s[j])) j++;
    if (j != b || end - a >= sizeof buf) return ING_ERR;
    memcpy(buf, s + a, end - a);
    buf[end - a] = 0;
    *out = strtod(buf, NULL); /* glibc: correctly rounded, ties to even; saturates like Java */
    return ING_OK;
}

/* Long.valueOf(String): [+-]?digits, no trim, range-checked */
static int j_parse_long(const char* s, size_t n, int64_t* out) {
    if (n == 0) return ING_ERR;
    size_t i = 0;
    int neg = 0;
    if (s[0] == '+' || s[0] == '-') {
        neg = s[0] == '-';
        i = 1;
    }
    if (i == n) return ING_ERR;
    __int128 v = 0;
    for (; i < n; i++) {
        if (!isdig(s[i])) return ING_ERR;
        v = v * 10 + (s[i] - '0');
        if (v > ((__int128)1 << 63)) return ING_ERR;
    }
    if (neg) v = -v;
    if (v > INT64_MAX || v < INT64_MIN) return ING_ERR;
    *out = (int64_t)v;
    return ING_OK;
}

/* str.replace("\"", "").split("\\s*" + delimiter + "\\s*") for a one-character delimiter that
   is not a regex metacharacter.  Field f of the split -> [*fs, *fe) in the quote-free copy t. */
static int j_csv_field(const char* t, size_t n, unsigned char d, int want, size_t* fs, size_t* fe) {
    /* find separator matches left to right */
    size_t starts[4096], ends[4096];
    int nf = 0;
    size_t cur = 0;
    size_t i = 0;
    while (i < n) {
        /* leftmost match at i: \s* then d then \s*.  Non-space d: the first non-\s at or after i
           must be d.  Space d: the maximal \s run starting at i must contain d. */
        size_t j = i, k;
        int hit = 0;
        if (!jspace(d)) {
            while (j < n && jspace((unsigned char)t[j])) j++;
            if (j < n && (unsigned char)t[j] == d) {
                hit = 1;
                k = j + 1;
                while (k < n && jspace((unsigned char)t[k])) k++;
            }
        } else if (jspace((unsigned char)t[i])) {
            int has = 0;
            while (j < n && jspace((unsigned char)t[j])) has |= (unsigned char)t[j] == d, j++;
            if (has) {
                hit = 1;
                k = j;
            }
        }
        if (!hit) {
            i++;
            continue;
        }
        if (nf >= 4095) return ING_ERR;
        starts[nf] = cur;
        ends[nf] = i;
        nf++;
        cur = k;
        i = k;
    }
    starts[nf] = cur;
    ends[nf] = n;
    nf++;
    while (nf > 0 && starts[nf - 1] == ends[nf - 1]) nf--; /* trailing empty strings removed */
    if (nf == 0) nf = 1, starts[0] = ends[0] = 0;          /* "".split(..) -> [""] */
    if (want < 0 || want >= nf) return ING_ERR;            /* IndexOutOfBoundsException */
    *fs = starts[want];
    *fe = ends[want];
    return ING_OK;
}

/* oid (nullable): CSVTSVToTSpatial's strOId = strArrayList.get(csvTsvSchemaAttr.get(0)),
   Deserialization.java:313-314 -- copied out of the quote-free record into *oidbuf (malloc'd). */
static int csv_record(const char* r, size_t n, const ing_spec* sp, double* x, double* y, int64_t* ts,
                      ing_oid* oid, char** oidbuf) {
    char* t = (char*)malloc(n + 1);
    size_t m = 0;
    for (size_t i = 0; i < n; i++)
        if (r[i] != '"') t[m++] = r[i];
    size_t a, b;
    int rc = ING_OK;
    /* CSVTSVToTSpatial evaluates get(0), then Long.valueOf(get(1)), then x, then y */
    if (oid && sp->foid >= 0) {
        rc = j_csv_field(t, m, (unsigned char)sp->delim, sp->foid, &a, &b);
        if (!rc) {
            /* libgeohip restates non-empty objIDs without control characters (other than \s) */
            if (a == b) rc = ING_UNDECIDED;
            for (size_t i = a; !rc && i < b; i++)
                if ((unsigned char)t[i] < 0x20 && !jspace((unsigned char)t[i])) rc = ING_UNDECIDED;
        }
        if (!rc) {
            *oidbuf = (char*)malloc(b - a + 1);
            memcpy(*oidbuf, t + a, b - a);
            oid->null = 0;
            oid->buf = *oidbuf;
            oid->a = 0;
            oid->b = b - a;
        }
    }
    if (!rc && sp->fts >= 0) {
        rc = j_csv_field(t, m, (unsigned char)sp->delim, sp->fts, &a, &b);
        if (!rc) rc = j_parse_long(t + a, b - a, ts);
    }
    if (!rc) rc = j_csv_field(t, m, (unsigned char)sp->delim, sp->fx, &a, &b);
    if (!rc) rc = j_parse_double(t + a, b - a, x);
    if (!rc) rc = j_csv_field(t, m, (unsigned char)sp->delim, sp->fy, &a, &b);
    if (!rc) rc = j_parse_double(t + a, b - a, y);
    free(t);
    return rc;
}

/* ---- GeoJSON: a small strict JSON reader (Jackson grammar) ------------------------------ */
typedef struct {
    const char* s;
    size_t n, p;
} jr;

static void jws(jr* r) {
    while (r->p < r->n && (r->s[r->p] == ' ' || r->s[r->p] == '\t' || r->s[r->p] == '\r' || r->s[r->p] == '\n')) r->p++;
}
static int jskip(jr* r, int depth);
static int jstring(jr* r, size_t* a, size_t* b) {
    if (r->p >= r->n || r->s[r->p] != '"') return ING_ERR;
    r->p++;
    *a = r->p;
    while (r->p < r->n && r->s[r->p] != '"') {
        if ((unsigned char)r->s[r->p] < 0x20) return ING_ERR;
        if (r->s[r->p] == '\\') r->p++;
        r->p++;
    }
    if (r->p >= r->n) return ING_ERR;
    *b = r->p++;
    return ING_OK;
}
/* JSON number token -> the double JTS finally sees: Jackson DoubleNode (Double.parseDouble),
   or an IntNode/LongNode for integer tokens ("-0" -> 0), re-serialised and re-read exactly. */
static int jnumber(jr* r, double* out) {
    size_t a = r->p, i = a;
    const char* s = r->s;
    if (i < r->n && s[i] == '-') i++;
    size_t d0 = i;
    while (i < r->n && isdig(s[i])) i++;
    size_t ni = i - d0;
    if (ni == 0 || (ni > 1 && s[d0] == '0')) return ING_ERR;
    int isint = 1;
    if (i < r->n && s[i] == '.') {
        isint = 0;
        i++;
        size_t f0 = i;
        while (i < r->n && isdig(s[i])) i++;
        if (i == f0) return ING_ERR;
    }
    if (i < r->n && (s[i] == 'e' || s[i] == 'E')) {
        isint = 0;
        i++;
        if (i < r->n && (s[i] == '+' || s[i] == '-')) i++;
        size_t e0 = i;
        while (i < r->n && isdig(s[i])) i++;
        if (i == e0) return ING_ERR;
    }
    char buf[512];
    if (i - a >= sizeof buf) return ING_ERR;
    memcpy(buf, s + a, i - a);
    buf[i - a] = 0;
    r->p = i;
    if (isint) {
        int64_t v;
        if (j_parse_long(buf, i - a, &v)) return ING_ERR; /* BigIntegerNode: not followed here */
        *out = (double)v;                                 /* long -> double, round to nearest */
        return ING_OK;
    }
    *out = strtod(buf, NULL);
    return isinf(*out) ? ING_ERR : ING_OK; /* DoubleNode(Infinity) -> "Infinity": not JSON */
}
static int jskip(jr* r, int depth) {
    if (depth > 64) return ING_ERR;
    jws(r);
    if (r->p >= r->n) return ING_ERR;
    char c = r->s[r->p];
    size_t a, b;
    double v;
    if (c == '"') return jstring(r, &a, &b);
    if (c == '{' || c == '[') {
        char close = c == '{' ? '}' : ']';
        r->p++;
        jws(r);
        if (r->p < r->n && r->s[r->p] == close) {
            r->p++;
            return ING_OK;
        }
        for (;;) {
            if (c == '{') {
                jws(r);
                if (jstring(r, &a, &b)) return ING_ERR;
                jws(r);
                if (r->p >= r->n || r->s[r->p] != ':') return ING_ERR;
                r->p++;
            }
            if (jskip(r, depth + 1)) return ING_ERR;
            jws(r);
            if (r->p >= r->n) return ING_ERR;
            if (r->s[r->p] == ',') {
                r->p++;
                continue;
            }
            if (r->s[r->p] == close) {
                r->p++;
                return ING_OK;
            }
            return ING_ERR;
        }
    }
    if (c == '-' || isdig(c)) return jnumber(r, &v);
    static const char* lits[] = {"true", "false", "null"};
    for (int k = 0; k < 3; k++) {
        size_t L = strlen(lits[k]);
        if (r->n - r->p >= L && memcmp(r->s + r->p, lits[k], L) == 0) {
            r->p += L;
            return ING_OK;
        }
    }
    return ING_ERR;
}
/* object at r->p: position of the value of member `key` (last one wins, like ObjectNode) */
static int jmember(const char* s, size_t n, size_t obj, const char* key, size_t* at) {
    jr r = {s, n, obj};
    jws(&r);
    if (r.p >= n || s[r.p] != '{') return ING_ERR;
    r.p++;
    int found = 0;
    jws(&r);
    if (r.p < n && s[r.p] == '}') return ING_ERR;
    for (;;) {
        size_t a, b;
        jws(&r);
        if (jstring(&r, &a, &b)) return ING_ERR;
        jws(&r);
        if (r.p >= n || s[r.p] != ':') return ING_ERR;
        r.p++;
        jws(&r);
        if (b - a == strlen(key) && memcmp(s + a, key, b - a) == 0) {
            *at = r.p;
            found = 1;
        }
        if (jskip(&r, 1)) return ING_ERR;
        jws(&r);
        if (r.p < n && s[r.p] == ',') {
            r.p++;
            continue;
        }
        if (r.p < n && s[r.p] == '}') break;
        return ING_ERR;
    }
    return found ? ING_OK : ING_ERR;
}
/* geometry.getCoordinate(): the first position of the (nested) coordinates array */
static int geojson_record(const char* s, size_t n, double* x, double* y) {
    jr whole = {s, n, 0};
    if (jskip(&whole, 0)) return ING_ERR; /* the Kafka value must be valid JSON */
    size_t at;
    /* readGeoJSON(value): a geometry object carries "coordinates"; otherwise (Feature) the
       reader throws and value.geometry is read instead (Deserialization.java:134-141) */
    if (jmember(s, n, 0, "coordinates", &at)) {
        size_t g;
        if (jmember(s, n, 0, "geometry", &g)) return ING_ERR;
        if (jmember(s, n, g, "coordinates", &at)) return ING_ERR;
    }
    jr r = {s, n, at};
    jws(&r);
    if (r.p >= n || s[r.p] != '[') return ING_ERR;
    while (r.p < n && s[r.p] == '[') {
        r.p++;
        jws(&r);
    }
    if (jnumber(&r, x)) return ING_ERR;
    jws(&r);
    if (r.p >= n || s[r.p] != ',') return ING_ERR;
    r.p++;
    jws(&r);
    if (jnumber(&r, y)) return ING_ERR;
    return ING_OK;
}

/* ---- GeoJSONToTSpatial (Deserialization.java:149-208) -------------------------------------- */
/* the keys of the object at obj hold no backslash (libgeohip compares keys as written) */
static int jkeys_plain(const char* s, size_t n, size_t obj) {
    jr r = {s, n, obj};
    jws(&r);
    if (r.p >= n || s[r.p] != '{') return 1;
    r.p++;
    jws(&r);
    if (r.p < n && s[r.p] == '}') return 1;
    for (;;) {
        size_t a, b;
        jws(&r);
        if (jstring(&r, &a, &b)) return 0;
        if (memchr(s + a, '\\', b - a)) return 0;
        jws(&r);
        r.p++; /* ':' */
        if (jskip(&r, 1)) return 0;
        jws(&r);
        if (r.p < n && s[r.p] == ',') {
            r.p++;
            continue;
        }
        return 1;
    }
}

/* SimpleDateFormat("yyyy-MM-dd HH:mm:ss").parse(text) (lenient) then getTime() in a zone of fixed
   offset off_min.  Restated here: the 'yyyy-MM-dd HH:mm:ss' digit counts after blanks, year
   1583..9999, fields carried over by timegm's normalisation (the lenient calendar's arithmetic);
   no parse at all (ParseException, caught by the reference) -> 0.  Other forms -> ING_UNDECIDED. */
static int j_date_parse(const char* s, size_t n, int32_t off_min, int64_t* ms) {
    size_t i = 0;
    while (i < n && (s[i] == ' ' || s[i] == '\t')) i++;
    if (i == n) {
        *ms = 0;
        return ING_OK;
    }
    unsigned char c = (unsigned char)s[i];
    if (c < 0x80 && !isdig(c) && c != '-' && c != '+' && c != 'N') { /* DecimalFormat parses nothing */
        *ms = 0;
        return ING_OK;
    }
    const char* t = s + i;
    size_t L = n - i;
    static const int digit_at[] = {0, 1, 2, 3, 5, 6, 8, 9, 11, 12, 14, 15, 17, 18};
    if (L < 19 || t[4] != '-' || t[7] != '-' || t[10] != ' ' || t[13] != ':' || t[16] != ':') return ING_UNDECIDED;
    for (int k = 0; k < 14; k++)
        if (!isdig((unsigned char)t[digit_at[k]])) return ING_UNDECIDED;
    if (L > 19) {
        unsigned char e = (unsigned char)t[19];
        if (e >= 0x80 || isdig(e) || strchr("Ee.,", e)) return ING_UNDECIDED;
    }
    int Y = atoi((char[]){t[0], t[1], t[2], t[3], 0});
    if (Y < 1583) return ING_UNDECIDED;
    struct tm tm;
    memset(&tm, 0, sizeof tm);
    tm.tm_year = Y - 1900;
    tm.tm_mon = (t[5] - '0') * 10 + (t[6] - '0') - 1;
    tm.tm_mday = (t[8] - '0') * 10 + (t[9] - '0');
    tm.tm_hour = (t[11] - '0') * 10 + (t[12] - '0');
    tm.tm_min = (t[14] - '0') * 10 + (t[15] - '0');
    tm.tm_sec = (t[17] - '0') * 10 + (t[18] - '0');
    const time_t secs = timegm(&tm);
    *ms = ((int64_t)secs - (int64_t)off_min * 60) * 1000;
    return ING_OK;
}

static int geojson_traj_record(const char* s, size_t n, const ing_traj* tr, double* x, double* y, int64_t* ts,
                               ing_oid* oid) {
    int rc = geojson_record(s, n, x, y);
    if (rc) return rc;
    *ts = 0;
    oid->null = 1;
    if (!jkeys_plain(s, n, 0)) return ING_UNDECIDED;
    /* trailing text after the value: Jackson ignores it, libgeohip does not restate that */
    {
        jr w = {s, n, 0};
        jskip(&w, 0);
        jws(&w);
        if (w.p != n) return ING_UNDECIDED;
    }
    size_t props;
    if (jmember(s, n, 0, "properties", &props)) return ING_OK; /* nodeProperties == null */
    if (!jkeys_plain(s, n, props)) return ING_UNDECIDED;
    size_t at;
    if (tr->date_format != 0 && !jmember(s, n, props, tr->prop_ts, &at)) {
        /* dateFormat.parse(nodeTime.textValue()): a non-string node has no text -> NPE */
        jr r = {s, n, at};
        size_t a, b;
        if (s[at] != '"' || jstring(&r, &a, &b)) return ING_ERR;
        if (memchr(s + a, '\\', b - a)) return ING_UNDECIDED;
        rc = j_date_parse(s + a, b - a, tr->utc_offset_min, ts);
        if (rc) return rc;
    }
    if (!jmember(s, n, props, tr->prop_oid, &at)) {
        /* nodeOId.toString().replaceAll("\"", ""): Jackson's text of the node, quotes deleted */
        jr r = {s, n, at};
        size_t a = at, b;
        if (s[at] == '"') {
            size_t sa, sb;
            if (jstring(&r, &sa, &sb)) return ING_ERR;
            for (size_t i = sa; i < sb; i++)
                if ((unsigned char)s[i] < 0x20 || (unsigned char)s[i] >= 0x7f || s[i] == '\\') return ING_UNDECIDED;
            a = sa;
            b = sb;
        } else {
            if (jskip(&r, 1)) return ING_ERR;
            b = r.p;
            int lit = (b - a == 4 && !memcmp(s + a, "true", 4)) || (b - a == 5 && !memcmp(s + a, "false", 5)) ||
                      (b - a == 4 && !memcmp(s + a, "null", 4));
            int integer = b > a && (isdig((unsigned char)s[a]) || s[a] == '-');
            for (size_t i = a + (s[a] == '-'); integer && i < b; i++) integer = isdig((unsigned char)s[i]);
            if (integer && b - a == 2 && s[a] == '-' && s[a + 1] == '0') integer = 0; /* IntNode(0): "0" */
            if (!lit && !integer) return ING_UNDECIDED;
        }
        oid->null = 0;
        oid->buf = s;
        oid->a = a;
        oid->b = b;
    }
    return ING_OK;
}

/* ---- WKT: JTS WKTReader on str.substring(str.indexOf("POINT")) ----------------------------- */
static int wword(unsigned char c) {
    return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || isdig(c) || c == '-' || c == '+' || c == '.' || c >= 160;
}
/* StreamTokenizer: next token as [a, b); ordinary chars are one-char tokens; '#' comments */
static int wtok(const char* s, size_t n, size_t* p, size_t* a, size_t* b) {
    for (;;) {
        while (*p < n && (unsigned char)s[*p] <= ' ') (*p)++;
        if (*p < n && s[*p] == '#') {
            while (*p < n && s[*p] != '\n' && s[*p] != '\r') (*p)++;
            continue;
        }
        break;
    }
    if (*p >= n) return 0;
    *a = *p;
    if (wword((unsigned char)s[*p])) {
        while (*p < n && wword((unsigned char)s[*p])) (*p)++;
    } else {
        (*p)++;
    }
    *b = *p;
    return 1;
}
static int wkt_number(const char* s, size_t a, size_t b, double* v) {
    if (b - a == 3 && strncasecmp(s + a, "NaN", 3) == 0) { /* WKTReader.getNextNumber */
        *v = NAN;
        return ING_OK;
    }
    if (!wword((unsigned char)s[a])) return ING_ERR;
    return j_parse_double(s + a, b - a, v);
}
static int wkt_record(const char* s, size_t n, double* x, double* y) {
    size_t pos = 0;
    int found = 0;
    for (; pos + 5 <= n; pos++)
        if (memcmp(s + pos, "POINT", 5) == 0) {
            found = 1;
            break;
        }
    if (!found) return ING_ERR; /* substring(-1): StringIndexOutOfBoundsException */
    size_t p = pos, a, b;
    if (!wtok(s, n, &p, &a, &b) || b - a != 5) return ING_ERR; /* "POINT" as a whole word */
    if (!wtok(s, n, &p, &a, &b) || s[a] != '(' || b - a != 1) return ING_ERR; /* EMPTY, Z, M: not here */
    if (!wtok(s, n, &p, &a, &b) || wkt_number(s, a, b, x)) return ING_ERR;
    if (!wtok(s, n, &p, &a, &b) || wkt_number(s, a, b, y)) return ING_ERR;
    if (!wtok(s, n, &p, &a, &b)) return ING_ERR;
    if (s[a] == ')' && b - a == 1) return ING_OK;
    double z; /* a third ordinate is read and dropped by getCoordinate() x/y */
    if (wkt_number(s, a, b, &z)) return ING_ERR;
    if (!wtok(s, n, &p, &a, &b) || s[a] != ')' || b - a != 1) return ING_ERR;
    return ING_OK;
}

static int32_t j_d2i(double v) {
    if (v != v) return 0;
    if (v >= 2147483647.0) return INT32_MAX;
    if (v <= -2147483648.0) return INT32_MIN;
    return (int32_t)v;
}

static int any_record(const ing_spec* sp, const ing_traj* tr, const char* r, size_t n, double* x, double* y,
                      int64_t* ts, ing_oid* oid, char** oidbuf) {
    *ts = 0;
    if (oid) oid->null = 1;
    if (sp->format == FMT_CSV) return csv_record(r, n, sp, x, y, ts, oid, oidbuf);
    if (sp->format == FMT_GEOJSON) return tr ? geojson_traj_record(r, n, tr, x, y, ts, oid) : geojson_record(r, n, x, y);
    return wkt_record(r, n, x, y); /* WKTToTSpatial: objID null, timestamp 0 */
}

/* One record -> (x, y, ts, cell).  cell = cx * n + cy for a valid key, else 0xffffffff. */
int geohip_oracle_ingest_record(const ing_spec* sp, const ing_grid* g, const char* r, size_t n, double* x,
                                double* y, int64_t* ts, uint32_t* cell) {
    int rc = any_record(sp, NULL, r, n, x, y, ts, NULL, NULL);
    if (rc) return rc;
    const int32_t cx = j_d2i(floor((*x - g->min_x) / g->cell_len));
    const int32_t cy = j_d2i(floor((*y - g->min_y) / g->cell_len));
    *cell = (cx >= 0 && cx < g->n && cy >= 0 && cy < g->n) ? (uint32_t)cx * (uint32_t)g->n + (uint32_t)cy : 0xffffffffu;
    return ING_OK;
}

/* A text batch: records split at '\n'.  Returns the record count, or -(1 + i) for the first
   record i the reference rejects; cap bounds the outputs. */
int64_t geohip_oracle_ingest(const ing_spec* sp, const ing_grid* g, const char* text, uint64_t nbytes, double* x,
                             double* y, int64_t* ts, uint32_t* cell, uint64_t cap) {
    uint64_t p = 0, rec = 0;
    while (p < nbytes) {
        const char* nl = memchr(text + p, '\n', nbytes - p);
        uint64_t e = nl ? (uint64_t)(nl - text) : nbytes;
        double xv, yv;
        int64_t tv;
        uint32_t cv;
        if (geohip_oracle_ingest_record(sp, g, text + p, e - p, &xv, &yv, &tv, &cv)) return -(int64_t)(rec + 1);
        if (rec < cap) {
            x[rec] = xv;
            y[rec] = yv;
            if (ts) ts[rec] = tv;
            if (cell) cell[rec] = cv;
        }
        rec++;
        p = e + 1;
    }
    return (int64_t)rec;
}

/* TrajectoryStream batch (CSVTSVToTSpatial / GeoJSONToTSpatial / WKTToTSpatial): as
   geohip_oracle_ingest plus the objID strings -- oid_buf (oid_cap bytes) and oid_off[rec + 1]
   (bit 63: null objID).  Returns the record count, -(1 + i) for the first record i rejected
   (thrown or not restated), or INT64_MIN when oid_cap is too small. */
int64_t geohip_oracle_ingest_traj(const ing_spec* sp, const ing_traj* tr, const ing_grid* g, const char* text,
                                  uint64_t nbytes, double* x, double* y, int64_t* ts, uint32_t* cell, char* oid_buf,
                                  uint64_t oid_cap, uint64_t* oid_off, uint64_t cap) {
    uint64_t p = 0, rec = 0, ob = 0;
    while (p < nbytes) {
        const char* nl = memchr(text + p, '\n', nbytes - p);
        uint64_t e = nl ? (uint64_t)(nl - text) : nbytes;
        double xv, yv;
        int64_t tv;
        ing_oid oid = {1, NULL, 0, 0};
        char* own = NULL;
        int rc = any_record(sp, sp->format == FMT_GEOJSON ? tr : NULL, text + p, e - p, &xv, &yv, &tv, &oid, &own);
        if (rc) {
            free(own);
            return -(int64_t)(rec + 1);
        }
        if (rec < cap) {
            x[rec] = xv;
            y[rec] = yv;
            ts[rec] = tv;
            const int32_t cx = j_d2i(floor((xv - g->min_x) / g->cell_len));
            const int32_t cy = j_d2i(floor((yv - g->min_y) / g->cell_len));
            cell[rec] = (cx >= 0 && cx < g->n && cy >= 0 && cy < g->n) ? (uint32_t)cx * (uint32_t)g->n + (uint32_t)cy
                                                                       : 0xffffffffu;
            oid_off[rec] = ob | (oid.null ? 1ull << 63 : 0ull);
            if (!oid.null) {
                for (size_t i = oid.a; i < oid.b; i++) {
                    if (oid.buf[i] == '"') continue;
                    if (ob >= oid_cap) {
                        free(own);
                        return INT64_MIN;
                    }
                    oid_buf[ob++] = oid.buf[i];
                }
            }
        }
        free(own);
        rec++;
        p = e + 1;
    }
    if (rec <= cap) oid_off[rec] = ob;
    return (int64_t)rec;
}
