/*
 * The Scala half of the seam: the binding a maintainer adds to the reference
 * (core/src/main/scala/org/apache/spark/sql/delta/gpu/) next to jni/deltareplay_jni.c. Source only --
 * this image has no JVM or scalac; INTEGRATION.md §1 shows where Snapshot calls it.
 *
 * D/ = core/src/main/scala/org/apache/spark/sql/delta/.
 */
package org.apache.spark.sql.delta.gpu

import java.nio.{ByteBuffer, ByteOrder}
import java.nio.charset.StandardCharsets.UTF_8

import org.apache.spark.sql.delta.actions.{AddFile, RemoveFile}

object DeltaReplayNative {
  System.loadLibrary("deltareplay_jni")   // links libdeltareplay.so

  /** include/deltareplay.h DR_ABI_VERSION this binding was written against. */
  val AbiVersion = 4
  require(abiVersion() == AbiVersion,
    s"libdeltareplay ABI ${abiVersion()} does not match the binding's $AbiVersion")

  @native def abiVersion(): Int
  @native def ctxCreate(device: Int): Long
  @native def ctxDestroy(ctx: Long): Unit
  /** dr_ctx_set_option (ABI 4): one of the Opt* options below, set from the session's conf. */
  @native def setOption(ctx: Long, option: Int, value: Long): Unit
  val OptOverlap = 1; val OptSplit = 2; val OptBucketBits = 3; val OptFilterEval = 4; val OptApplyFull = 5
  val OptCanonHint = 6; val OptJsonStaged = 7; val OptHostCacheBytes = 8
  // Text crosses the boundary as UTF-8 bytes (the *Utf8 natives): JNI's string calls use modified
  // UTF-8, which would corrupt characters outside the BMP in table paths and metaData values. The
  // String-typed methods below convert with StandardCharsets.UTF_8.
  @native def lastErrorUtf8(ctx: Long): Array[Byte]
  @native def stageLogUtf8(ctx: Long, logPath: Array[Byte], version: Long): Long
  @native def stageLogShardUtf8(ctx: Long, logPath: Array[Byte], version: Long, world: Int, rank: Int): Long
  @native def stage(ctx: Long, versions: Array[Long], bytes: Array[Array[Byte]]): Long
  @native def stageNamedUtf8(ctx: Long, logPath: Array[Byte], versions: Array[Long], kinds: Array[Int],
                             parts: Array[Int], names: Array[Array[Byte]], bytes: Array[Array[Byte]]): Long
  @native def stagedRelease(staged: Long): Unit
  @native def replay(ctx: Long, staged: Long, minFileRetentionTs: Long, validate: Boolean): Long
  /** 0 = DR_E_REBUILD: replay the new segment instead. */
  @native def apply(ctx: Long, state: Long, tail: Long, minFileRetentionTs: Long, validate: Boolean): Long
  @native def release(state: Long): Unit
  @native def counts(state: Long): Array[Long]
  @native def localCounts(state: Long): Array[Long]
  @native def nonFileJsonUtf8(state: Long): Array[Byte]
  @native def setNonFileJsonUtf8(state: Long, lines: Array[Byte], validate: Boolean): Unit
  /** null: the counters match (or there is no readable .crc); else checkMismatch's text. */
  @native def checkChecksumUtf8(state: Long, crcLine: Array[Byte]): Array[Byte]
  @native def recordSums(state: Long): Array[Long]
  /** A whole side; UnsupportedOperationException when a column exceeds a direct buffer (2^31 - 1
   *  bytes): take it as ranges instead. */
  @native def export(state: Long, which: Int): Array[ByteBuffer]
  /** Row boundaries {0, ..., n} of ranges of at most maxRows rows and maxBytes bytes per column (ABI 3). */
  @native def exportPlan(state: Long, which: Int, maxRows: Long, maxBytes: Long): Array[Long]
  /** Rows [lo, hi) with offsets rebased to the range; handleOut(0) receives the range, freed with
   *  rangeRelease (independent of the state). */
  @native def exportRange(state: Long, which: Int, lo: Long, hi: Long, handleOut: Array[Long]): Array[ByteBuffer]
  @native def rangeRelease(range: Long): Unit
  @native def filter(state: Long, program: Array[Byte]): Array[Long]
  @native def scanOrder(state: Long): Array[Long]
  @native def partitionGroups(state: Long, rows: Array[Long]): Array[Array[Long]]
  /** dr_lines' columns; handleOut(0) receives the parse to release with parsedRelease. */
  @native def parseCommits(ctx: Long, staged: Long, handleOut: Array[Long]): Array[ByteBuffer]
  @native def parsedRelease(parsed: Long): Unit
  @native def commUniqueId(): Array[Byte]
  @native def commCreate(ctx: Long, id: Array[Byte], world: Int, rank: Int): Long
  @native def commRelease(comm: Long): Unit
  @native def replaySharded(comm: Long, staged: Long, minFileRetentionTs: Long, validate: Boolean): Long
  @native def writeCheckpoint(state: Long, part: Int, parts: Int, opts: Int, rowGroupRows: Long,
                              rowsOut: Array[Long]): Array[Byte]

  val Live = 0
  val Tombstones = 1
  /** The largest column a direct ByteBuffer can hold. */
  val MaxBufferBytes: Long = Int.MaxValue.toLong

  private def utf8(b: Array[Byte]): String = if (b == null) null else new String(b, UTF_8)
  def lastError(ctx: Long): String = utf8(lastErrorUtf8(ctx))
  def stageLog(ctx: Long, logPath: String, version: Long): Long = stageLogUtf8(ctx, logPath.getBytes(UTF_8), version)
  def stageLogShard(ctx: Long, logPath: String, version: Long, world: Int, rank: Int): Long =
    stageLogShardUtf8(ctx, logPath.getBytes(UTF_8), version, world, rank)
  def stageNamed(ctx: Long, logPath: String, versions: Array[Long], kinds: Array[Int], parts: Array[Int],
                 names: Array[String], bytes: Array[Array[Byte]]): Long =
    stageNamedUtf8(ctx, logPath.getBytes(UTF_8), versions, kinds, parts, names.map(_.getBytes(UTF_8)), bytes)
  def nonFileJson(state: Long): String = utf8(nonFileJsonUtf8(state))
  def setNonFileJson(state: Long, lines: String, validate: Boolean): Unit =
    setNonFileJsonUtf8(state, lines.getBytes(UTF_8), validate)
  def checkChecksum(state: Long, crcLine: Array[Byte]): String = utf8(checkChecksumUtf8(state, crcLine))

  /** Order of counts() / localCounts() (dr_counts). */
  object CountFields {
    val NumFiles = 0; val SizeInBytes = 1; val NumRemoves = 2; val NumMetadata = 3; val NumProtocol = 4
    val NumSetTransactions = 5; val NumActions = 6; val NumFileActions = 7; val Version = 8
    val MalformedLines = 9; val LiveKeySum = 10; val TombKeySum = 11
  }

  /** Indices of export()'s buffers (dr_export's columns in declaration order). */
  object ExportColumns {
    val PathOff = 0; val PathBytes = 1; val Size = 2; val ModificationTime = 3; val DeletionTimestamp = 4
    val DeletionTimestampValid = 5; val ExtendedFileMetadata = 6; val StatsOff = 7; val StatsBytes = 8
    val StatsNull = 9; val PvEntryOff = 10; val PvNull = 11; val PvKeyOff = 12; val PvKeyBytes = 13
    val PvValOff = 14; val PvValBytes = 15; val PvValNull = 16; val TagsEntryOff = 17; val TagsNull = 18
    val TagsKeyOff = 19; val TagsKeyBytes = 20; val TagsValOff = 21; val TagsValBytes = 22; val TagsValNull = 23
  }

  /** A lowered partition predicate (dr_predicate), serialised as filter() reads it. Opcodes and type
   *  codes are include/deltareplay.h's dr_pred_opcode / dr_pred_type. */
  final case class Program(ops: Seq[(Int, Int)], cols: Seq[(String, Int)],
                           lits: Seq[(Int, Boolean, Long, Array[Byte])]) {
    def serialize: Array[Byte] = {
      val size = 4 + 8 * ops.size + 4 + cols.map(c => 8 + c._1.getBytes(UTF_8).length).sum +
        4 + lits.map(l => 17 + l._4.length).sum
      val b = ByteBuffer.allocate(size).order(ByteOrder.LITTLE_ENDIAN)
      b.putInt(ops.size); ops.foreach { case (op, arg) => b.putInt(op).putInt(arg) }
      b.putInt(cols.size)
      cols.foreach { case (name, t) => val n = name.getBytes(UTF_8); b.putInt(t).putInt(n.length).put(n) }
      b.putInt(lits.size)
      lits.foreach { case (t, isNull, v, s) =>
        b.putInt(t).put((if (isNull) 1 else 0).toByte).putLong(v).putInt(s.length).put(s) }
      b.array()
    }
  }
}

/**
 * allFiles / tombstones from export()'s columns (D/Snapshot.scala:193-204): the reference's own
 * AddFile / RemoveFile case classes, dataChange = false as InMemoryLogReplay.checkpoint sets it
 * (D/actions/InMemoryLogReplay.scala:55-77), maps rebuilt from the entry offsets (a null map stays
 * null, a null value stays null), stats as the raw JSON string (@JsonRawValue). The buffers are read
 * in place (direct, little-endian); the rows copy what they keep, so the state may be released
 * afterwards.
 */
object SingleActionColumns {
  import DeltaReplayNative.ExportColumns._

  private def le(b: ByteBuffer): ByteBuffer = b.duplicate().order(ByteOrder.LITTLE_ENDIAN)

  // Offsets stay Long until a slice is taken; Math.toIntExact refuses (instead of wrapping) any
  // position a direct buffer cannot address -- the library's plan keeps every column of a range
  // under MaxBufferBytes, so it never fires on planned ranges.
  private final class Strings(off: ByteBuffer, bytes: ByteBuffer, nulls: ByteBuffer) {
    private val o = if (off == null) null else le(off)
    private val d = if (bytes == null) null else bytes.duplicate()
    def apply(i: Int): String = {
      if (o == null || (nulls != null && nulls.get(i) != 0)) return null
      val lo: Long = o.getLong(Math.toIntExact(8L * i))
      val hi: Long = o.getLong(Math.toIntExact(8L * i + 8))
      val a = new Array[Byte](Math.toIntExact(hi - lo))
      d.position(Math.toIntExact(lo)); d.get(a)
      new String(a, UTF_8)
    }
  }

  private final class Maps(c: Array[ByteBuffer], entryOff: Int, mapNull: Int, keyOff: Int, keyBytes: Int,
                           valOff: Int, valBytes: Int, valNull: Int) {
    private val eo = if (c(entryOff) == null) null else le(c(entryOff))
    private val keys = new Strings(c(keyOff), c(keyBytes), null)
    private val vals = new Strings(c(valOff), c(valBytes), c(valNull))
    def apply(i: Int): Map[String, String] = {
      if (eo == null || c(mapNull).get(i) != 0) return null
      val lo: Long = eo.getLong(Math.toIntExact(8L * i))
      val hi: Long = eo.getLong(Math.toIntExact(8L * i + 8))
      (lo until hi).map(e => keys(Math.toIntExact(e)) -> vals(Math.toIntExact(e))).toMap
    }
  }

  def rows(c: Array[ByteBuffer]): Int = (c(PathOff).capacity() / 8 - 1)

  def addFiles(c: Array[ByteBuffer]): Array[AddFile] = addFileIterator(c).toArray
  def removeFiles(c: Array[ByteBuffer]): Array[RemoveFile] = removeFileIterator(c).toArray

  /** The rows of one export (or range) lazily, for a partition iterator. */
  def addFileIterator(c: Array[ByteBuffer]): Iterator[AddFile] = {
    val n = rows(c)
    val path = new Strings(c(PathOff), c(PathBytes), null)
    val stats = new Strings(c(StatsOff), c(StatsBytes), c(StatsNull))
    val pv = new Maps(c, PvEntryOff, PvNull, PvKeyOff, PvKeyBytes, PvValOff, PvValBytes, PvValNull)
    val tags = new Maps(c, TagsEntryOff, TagsNull, TagsKeyOff, TagsKeyBytes, TagsValOff, TagsValBytes, TagsValNull)
    val size = le(c(Size)); val mtime = le(c(ModificationTime))
    Iterator.range(0, n).map { i =>
      AddFile(path(i), pv(i), size.getLong(8 * i), mtime.getLong(8 * i), dataChange = false, stats(i), tags(i))
    }
  }

  def removeFileIterator(c: Array[ByteBuffer]): Iterator[RemoveFile] = {
    val n = rows(c)
    val path = new Strings(c(PathOff), c(PathBytes), null)
    val pv = new Maps(c, PvEntryOff, PvNull, PvKeyOff, PvKeyBytes, PvValOff, PvValBytes, PvValNull)
    val tags = new Maps(c, TagsEntryOff, TagsNull, TagsKeyOff, TagsKeyBytes, TagsValOff, TagsValBytes, TagsValNull)
    val size = le(c(Size)); val dts = le(c(DeletionTimestamp))
    val dtsValid = c(DeletionTimestampValid); val efm = c(ExtendedFileMetadata)
    Iterator.range(0, n).map { i =>
      RemoveFile(path(i), if (dtsValid.get(i) != 0) Some(dts.getLong(8 * i)) else None, dataChange = false,
        extendedFileMetadata = efm.get(i) != 0, partitionValues = pv(i), size = size.getLong(8 * i),
        tags = tags(i))
    }
  }
}
