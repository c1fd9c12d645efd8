// ParityHarness.java -- decides SURVEY.md 8(c)'s open questions Q1-Q3 on a JVM with the reference.
//
// Source only: this image has no JDK (SURVEY.md 8(c)); the file is for the first maintainer who
// has one.  It reads tests/golden/jts_discriminators.json (made by tests/golden/make_discriminators.py)
// and runs every case through the reference's own distance functions -- the exact calls its
// operators make:
//   point-point   DistanceFunctions.getDistance(Point, Point)   (DistanceFunctions.java:15-18; the
//                 per-candidate distance of PointPointKNNQuery.java:95-98, 163-167 and of the
//                 range / join queries)
//   point-polygon DistanceFunctions.getDistance(Point, Polygon) (DistanceFunctions.java:33-36;
//                 PointPolygonRangeQuery.java:65, 116 and the point-polygon kNN / join)
// on Points and Polygons built by the reference's constructors (Point(double, double, UniformGrid),
// Polygon(List<List<Coordinate>>, UniformGrid), UniformGrid(int, double x4)).  For each question it
// prints how many cases follow reading A (what libgeohip and its oracle implement) and reading B,
// then one verdict line per question:  "Q1 A" means parity holds there; "Q1 B" names the
// restatement to change (oracle/restate.py, oracle/geohip_oracle.c, and the device functions in
// spatialflink_amd/csrc/device_common.h / cell_kernels.hip cited by tests/test_gpu_discriminators.py).
//
// The kNN case is decided by the same distances: the RealTime operator
// (PointPointKNNQuery.java:58-122, all points in one tumbling window, unique ids, no tie at rank k)
// returns the k smallest (distance, point) of its window, which the harness forms by sorting.
//
// Build and run (reference checked out at $REF, built once with `mvn -q -DskipTests package`):
//   CP=$(cd $REF && mvn -q dependency:build-classpath -Dmdep.outputFile=/dev/stdout):$REF/target/classes
//   javac -cp "$CP" -d /tmp/ph jvm/ParityHarness.java
//   java -cp "$CP:/tmp/ph" ParityHarness tests/golden/jts_discriminators.json
import GeoFlink.spatialIndices.UniformGrid;
import GeoFlink.spatialObjects.Point;
import GeoFlink.spatialObjects.Polygon;
import GeoFlink.utils.DistanceFunctions;
import org.json.JSONArray;
import org.json.JSONObject;
import org.locationtech.jts.geom.Coordinate;

import java.nio.charset.StandardCharsets;
import java.nio.file.Files;
import java.nio.file.Paths;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.Comparator;
import java.util.List;

public class ParityHarness {

    // float.hex strings ("0x1.d1a8f5c28f5c3p+6") are Java hex floating-point literals
    static double f(Object h) {
        return Double.parseDouble((String) h);
    }

    static long bits(double d) {
        return Double.doubleToRawLongBits(d);
    }

    static UniformGrid grid(JSONObject g) {
        return new UniformGrid(g.getInt("n"), f(g.get("min_x")), f(g.get("max_x")), f(g.get("min_y")), f(g.get("max_y")));
    }

    static Polygon polygon(JSONArray ring, UniformGrid g) {
        List<Coordinate> c = new ArrayList<>();
        for (int i = 0; i < ring.length(); i++) {
            JSONArray v = ring.getJSONArray(i);
            c.add(new Coordinate(f(v.get(0)), f(v.get(1))));
        }
        List<List<Coordinate>> rings = new ArrayList<>();
        rings.add(c);
        return new Polygon(rings, g);
    }

    static String verdict(int a, int b, int n) {
        if (a == n) return "A";
        if (b == n) return "B";
        return "mixed (A " + a + ", B " + b + ", neither " + (n - a - b) + ")";
    }

    public static void main(String[] args) throws Exception {
        String path = args.length > 0 ? args[0] : "tests/golden/jts_discriminators.json";
        JSONObject fx = new JSONObject(new String(Files.readAllBytes(Paths.get(path)), StandardCharsets.UTF_8));

        // ---- Q1: Coordinate.distance
        JSONObject q1 = fx.getJSONObject("Q1");
        JSONObject knn = q1.getJSONObject("knn");
        UniformGrid g1 = grid(knn.getJSONObject("grid"));
        JSONObject pq = q1.getJSONObject("pairs_from_query");
        JSONArray qv = pq.getJSONArray("query");
        Point q = new Point(f(qv.get(0)), f(qv.get(1)), g1);
        JSONArray cases = pq.getJSONArray("cases");
        int a = 0, b = 0;
        for (int i = 0; i < cases.length(); i++) {
            JSONObject c = cases.getJSONObject(i);
            JSONArray p = c.getJSONArray("p");
            double d = DistanceFunctions.getDistance(q, new Point(f(p.get(0)), f(p.get(1)), g1));
            if (bits(d) == bits(f(c.get("A")))) a++;
            else if (bits(d) == bits(f(c.get("B")))) b++;
        }
        System.out.println("Q1 pairs: A " + a + ", B " + b + " of " + cases.length());
        JSONArray xs = knn.getJSONArray("x"), ys = knn.getJSONArray("y");
        JSONArray kq = knn.getJSONArray("query");
        Point kqp = new Point(f(kq.get(0)), f(kq.get(1)), g1);
        final int n = xs.length();
        final double[] dist = new double[n];
        Integer[] order = new Integer[n];
        for (int i = 0; i < n; i++) {
            dist[i] = DistanceFunctions.getDistance(kqp, new Point(f(xs.get(i)), f(ys.get(i)), g1));
            order[i] = i;
        }
        Arrays.sort(order, Comparator.<Integer>comparingLong(i -> bits(dist[i])).thenComparingInt(i -> i));
        int k = knn.getInt("k");
        boolean knnA = true, knnB = true;
        JSONArray ia = knn.getJSONObject("A").getJSONArray("idx"), ib = knn.getJSONObject("B").getJSONArray("idx");
        for (int r = 0; r < k; r++) {
            knnA &= order[r] == ia.getInt(r);
            knnB &= order[r] == ib.getInt(r);
        }
        System.out.println("Q1 kNN window (k = " + k + "): A " + knnA + ", B " + knnB);
        System.out.println("VERDICT Q1 " + verdict(a + (knnA ? 1 : 0), b + (knnB ? 1 : 0), cases.length() + 1));

        // ---- Q2: RayCrossingCounter orientation (distance 0 inside / on the ring)
        JSONObject q2 = fx.getJSONObject("Q2");
        UniformGrid g2 = grid(q2.getJSONObject("grid"));
        Polygon poly2 = polygon(q2.getJSONArray("ring"), g2);
        JSONArray c2 = q2.getJSONArray("cases");
        a = 0;
        b = 0;
        for (int i = 0; i < c2.length(); i++) {
            JSONObject c = c2.getJSONObject(i);
            JSONArray p = c.getJSONArray("p");
            double d = DistanceFunctions.getDistance(new Point(f(p.get(0)), f(p.get(1)), g2), poly2);
            if (bits(d) == bits(f(c.get("A_dist")))) a++;
            else if (bits(d) == bits(f(c.get("B_dist")))) b++;
        }
        System.out.println("Q2 points by polygon edges: A " + a + ", B " + b + " of " + c2.length());
        System.out.println("VERDICT Q2 " + verdict(a, b, c2.length()));

        // ---- Q3: Distance.pointToSegment op order
        JSONObject q3 = fx.getJSONObject("Q3");
        UniformGrid g3 = grid(q3.getJSONObject("grid"));
        Polygon poly3 = polygon(q3.getJSONArray("ring"), g3);
        JSONArray c3 = q3.getJSONArray("cases");
        a = 0;
        b = 0;
        for (int i = 0; i < c3.length(); i++) {
            JSONObject c = c3.getJSONObject(i);
            JSONArray p = c.getJSONArray("p");
            double d = DistanceFunctions.getDistance(new Point(f(p.get(0)), f(p.get(1)), g3), poly3);
            if (bits(d) == bits(f(c.get("A")))) a++;
            else if (bits(d) == bits(f(c.get("B")))) b++;
        }
        System.out.println("Q3 exterior points: A " + a + ", B " + b + " of " + c3.length());
        System.out.println("VERDICT Q3 " + verdict(a, b, c3.length()));
    }
}
