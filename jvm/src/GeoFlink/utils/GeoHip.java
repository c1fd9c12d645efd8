// GeoHip.java -- the JNI facade over libgeohip.so that the drop-in operators
// (GeoFlink.spatialOperators.geohip.*) call once per window.  Source only here (no JDK in this
// image); jvm/build.sh builds it with jvm/native/geohip_jni.c against the reference's classpath.
//
// One native context per Flink task thread (include/geohip.h: a geohip_ctx is not shared between
// threads); windows cross the boundary as direct, native-order ByteBuffers of doubles (no GC
// pinning while the GPU works), results come back as window positions into the caller's list of
// Point objects, so the operators emit the very Point instances they received.
package GeoFlink.utils;

import GeoFlink.spatialIndices.UniformGrid;
import GeoFlink.spatialObjects.Point;
import GeoFlink.spatialObjects.Polygon;
import org.locationtech.jts.geom.Coordinate;
import org.locationtech.jts.geom.LineString;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.List;

public final class GeoHip implements AutoCloseable {
    static { System.loadLibrary("geohip_jni"); }  // libgeohip_jni.so, linked against libgeohip.so

    /** GEOHIP_ABI_VERSION of include/geohip.h this facade was written for. */
    public static final int ABI_VERSION = 2;

    private long ctx;  // geohip_ctx*

    /** A context on HIP device {@code device}; refuses a library of another ABI version. */
    public GeoHip(int device) {
        int v = abiVersion();
        if (v != ABI_VERSION)
            throw new IllegalStateException("libgeohip ABI " + v + ", facade written for " + ABI_VERSION);
        ctx = create(1 << device);
        // the window operators emit the hits as a set (PointPointRangeQuery.java:117-136): no
        // ordered emission (GEOHIP_ORDER_ANY = 1)
        rangeOrder(ctx, 1);
    }

    @Override
    public void close() {
        if (ctx != 0) {
            destroy(ctx);
            ctx = 0;
        }
    }

    /** geohip_grid from the UniformGrid getters (UniformGrid.java:136-146): both constructors. */
    public static double[] grid(UniformGrid g) {
        return new double[] {g.getMinX(), g.getMinY(), g.getCellLength(), g.getNumGridPartitions()};
    }

    /** A window's coordinates as two direct buffers: [0] = x, [1] = y. */
    public static ByteBuffer[] coords(List<Point> pts) {
        ByteBuffer x = doubles(pts.size()), y = doubles(pts.size());
        for (Point p : pts) {
            x.putDouble(p.point.getX());
            y.putDouble(p.point.getY());
        }
        return new ByteBuffer[] {x, y};
    }

    public static ByteBuffer doubles(int n) {
        return ByteBuffer.allocateDirect(8 * Math.max(n, 1)).order(ByteOrder.nativeOrder());
    }

    /** Rings of polygons as Polygon(List<List<Coordinate>>) built them (Polygon.java:115-165): for
     *  each polygon its JTS exterior ring, then its holes.  Returns {polyRings, ringOff} and fills
     *  vx / vy (the library closes open rings and takes the largest ring as the shell). */
    public static int[][] rings(List<Polygon> polys, List<Double> vx, List<Double> vy) {
        int[] polyRings = new int[polys.size() + 1];
        List<Integer> off = new ArrayList<>();
        off.add(0);
        for (int i = 0; i < polys.size(); i++) {
            org.locationtech.jts.geom.Polygon jp = polys.get(i).polygon;
            polyRings[i] = off.size() - 1;
            addRing(jp.getExteriorRing(), vx, vy, off);
            for (int h = 0; h < jp.getNumInteriorRing(); h++) addRing(jp.getInteriorRingN(h), vx, vy, off);
        }
        polyRings[polys.size()] = off.size() - 1;
        int[] ringOff = new int[off.size()];
        for (int j = 0; j < ringOff.length; j++) ringOff[j] = off.get(j);
        return new int[][] {polyRings, ringOff};
    }

    private static void addRing(LineString ring, List<Double> vx, List<Double> vy, List<Integer> off) {
        for (Coordinate c : ring.getCoordinates()) {
            vx.add(c.x);
            vy.add(c.y);
        }
        off.add(vx.size());
    }

    public static double[] unbox(List<Double> v) {
        double[] a = new double[v.size()];
        for (int i = 0; i < a.length; i++) a[i] = v.get(i);
        return a;
    }

    // ---- one call per window (include/geohip.h; the reference lines each replaces are cited there)

    /** geohip_range_pp: window positions of the hits, in no particular order (a set). */
    public int[] rangePP(double[] grid, ByteBuffer x, ByteBuffer y, int n, double qx, double qy, double r,
                         boolean approximate) {
        return rangePP(ctx, grid, x, y, n, qx, qy, r, approximate);
    }

    /** geohip_knn_pp: the min(k, candidates) nearest, ascending (distance, position); returns the count. */
    public int knnPP(double[] grid, ByteBuffer x, ByteBuffer y, int n, double qx, double qy, double r, int k,
                     int[] outIdx, double[] outDist) {
        return knnPP(ctx, grid, x, y, n, qx, qy, r, k, outIdx, outDist);
    }

    /** geohip_knn_range_pp: kNN (k) and range (r) of one query point in one pass; returns the kNN
     *  count, the range hits in the returned array's element [1]. */
    public int[][] knnRangePP(double[] grid, ByteBuffer x, ByteBuffer y, int n, double qx, double qy, double r,
                              int k, boolean approximate, int[] knnIdx, double[] knnDist) {
        return knnRangePP(ctx, grid, x, y, n, qx, qy, r, k, approximate, knnIdx, knnDist);
    }

    /** geohip_join_pp (two-phase): {dataPos, queryPos} pairs flattened, unordered. */
    public int[] joinPP(double[] gridData, double[] gridQuery, ByteBuffer dx, ByteBuffer dy, int nd, ByteBuffer qx,
                        ByteBuffer qy, int nq, double r, boolean approximate) {
        return joinPP(ctx, gridData, gridQuery, dx, dy, nd, qx, qy, nq, r, approximate);
    }

    /** geohip_range_ppoly (two-phase): {polygon, pointPos} pairs flattened, unordered. */
    public int[] rangePPoly(double[] grid, ByteBuffer x, ByteBuffer y, int n, int[] polyRings, int[] ringOff,
                            double[] vx, double[] vy, double r, boolean approximate) {
        return rangePPoly(ctx, grid, x, y, n, polyRings, ringOff, vx, vy, r, approximate);
    }

    /** geohip_join_ppoly (two-phase): {pointPos, polygon} pairs flattened, unordered. */
    public int[] joinPPoly(double[] uGrid, double[] qGrid, ByteBuffer x, ByteBuffer y, int n, int[] polyRings,
                           int[] ringOff, double[] vx, double[] vy, double r, boolean approximate) {
        return joinPPoly(ctx, uGrid, qGrid, x, y, n, polyRings, ringOff, vx, vy, r, approximate);
    }

    /** geohip_knn_ppoly: the nearest points of one polygon (its rings), ascending; returns the count. */
    public int knnPPoly(double[] grid, ByteBuffer x, ByteBuffer y, int n, int[] ringOff, double[] vx, double[] vy,
                        double r, int k, boolean approximate, int[] outIdx, double[] outDist) {
        return knnPPoly(ctx, grid, x, y, n, ringOff, vx, vy, r, k, approximate, outIdx, outDist);
    }

    private static native int abiVersion();
    private static native long create(int deviceMask);
    private static native void destroy(long ctx);
    private static native void rangeOrder(long ctx, int order);
    private static native int[] rangePP(long ctx, double[] g, ByteBuffer x, ByteBuffer y, int n, double qx, double qy,
                                        double r, boolean approx);
    private static native int knnPP(long ctx, double[] g, ByteBuffer x, ByteBuffer y, int n, double qx, double qy,
                                    double r, int k, int[] oi, double[] od);
    private static native int[][] knnRangePP(long ctx, double[] g, ByteBuffer x, ByteBuffer y, int n, double qx,
                                             double qy, double r, int k, boolean approx, int[] ki, double[] kd);
    private static native int[] joinPP(long ctx, double[] gd, double[] gq, ByteBuffer dx, ByteBuffer dy, int nd,
                                       ByteBuffer qx, ByteBuffer qy, int nq, double r, boolean approx);
    private static native int[] rangePPoly(long ctx, double[] g, ByteBuffer x, ByteBuffer y, int n, int[] polyRings,
                                           int[] ringOff, double[] vx, double[] vy, double r, boolean approx);
    private static native int[] joinPPoly(long ctx, double[] gu, double[] gq, ByteBuffer x, ByteBuffer y, int n,
                                          int[] polyRings, int[] ringOff, double[] vx, double[] vy, double r,
                                          boolean approx);
    private static native int knnPPoly(long ctx, double[] g, ByteBuffer x, ByteBuffer y, int n, int[] ringOff,
                                       double[] vx, double[] vy, double r, int k, boolean approx, int[] oi, double[] od);
}
