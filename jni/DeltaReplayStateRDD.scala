/*
 * Snapshot.state as a partitioned RDD over the GPU-resident replay (ABI 3 row ranges). Source only --
 * this image has no JVM or scalac; INTEGRATION.md §1 shows where Snapshot builds it.
 *
 * The reference keeps the reconstructed state as a partitioned Dataset (repartition into
 * snapshotPartitions, D/Snapshot.scala:103-110) cached MEMORY_AND_DISK_SER on the executors and
 * re-wrapped per session as a LogicalRDD (CachedDS, D/util/StateCache.scala:45-68). Here the state is
 * resident in HBM on the GPU that replayed it -- the driver's for a single-GPU replay, rank r's
 * executor for dr_replay_sharded -- and this RDD is its partitioned view: one partition per planned
 * row range (exportPlan: at most maxRows rows and 2^31 - 1 bytes per column, the JVM's direct-buffer
 * bound) of each rank's allFiles and tombstones, computed on the executor that holds the rank's state
 * (preferred location), pulling its rows with exportRange. No side is ever gathered on the driver, so
 * config 4's 100M-file state (36 GB of columns) crosses as ~2 GB slices.
 *
 * Recompute lineage (a single-GPU replay's partitions): the library lists a state's rows in the order
 * of their winning actions in the log segment (ABI 4, engine.hip:order_lists), so a row range is a
 * function of the segment and cutoff alone. A partition computed where its state is not resident --
 * scheduled off the replaying executor, or after that executor was lost -- replays the same segment
 * on this executor's GPU (the log's files are immutable) and exports the same rows, as the
 * reference's RDD recomputes from the log files. A sharded replay's rank state depends on the whole
 * exchange and cannot be rebuilt alone: its partitions still fail loudly off their executor.
 *
 * D/ = core/src/main/scala/org/apache/spark/sql/delta/.
 */
package org.apache.spark.sql.delta.gpu

import java.util.concurrent.ConcurrentHashMap

import org.apache.spark.{Partition, SparkContext, SparkEnv, TaskContext}
import org.apache.spark.rdd.RDD
import org.apache.spark.scheduler.ExecutorCacheTaskLocation
import org.apache.spark.sql.{Dataset, SparkSession}
import org.apache.spark.sql.catalyst.InternalRow
import org.apache.spark.sql.catalyst.encoders.ExpressionEncoder
import org.apache.spark.sql.delta.actions.SingleAction
import org.apache.spark.sql.execution.LogicalRDD

/**
 * One library context per GPU of this JVM, shared by every Snapshot and task on it (ABI 4: the library
 * serialises the calls that share a context). Options are the session's configuration of the path
 * (dr_ctx_set_option; the binding's Opt* constants), applied when the context is created.
 */
object DeltaReplayContexts {
  private val ctxs = new ConcurrentHashMap[Integer, java.lang.Long]()

  def forDevice(device: Int, options: Map[Int, Long] = Map.empty): Long =
    ctxs.computeIfAbsent(device, (d: Integer) => {
      val c = DeltaReplayNative.ctxCreate(d)
      options.foreach { case (k, v) => DeltaReplayNative.setOption(c, k, v) }
      java.lang.Long.valueOf(c)
    })
}

/**
 * Where a single-GPU replay's state comes from: enough to replay it again on another GPU (stageLog +
 * replay), plus the side sizes the rebuilt state must reproduce.
 */
final case class ReplaySource(logPath: String, version: Long, minFileRetentionTs: Long, validate: Boolean,
                              device: Int, numFiles: Long, numRemoves: Long)

/**
 * The states resident in this JVM, by (snapshot key, rank). A state is registered by the task that
 * replayed it and removed by Snapshot.uncache (D/util/StateCache.scala:104-109), which releases it.
 * Several tasks of one executor may export ranges of a state at once (the library serialises calls on
 * its context); every user holds a reference (`use`), and an uncache that arrives while tasks still
 * export only marks the state: the last user's return releases it (no call on a released state).
 */
object DeltaReplayStates {
  private final class Entry(val state: Long) {
    var users = 0
    var released = false
  }
  private val states = new ConcurrentHashMap[(String, Int), Entry]()
  private val rebuildLocks = new ConcurrentHashMap[String, Object]()
  /** Keys of states this JVM rebuilt, oldest first: at most `MaxRebuilt` stay resident (the driver's
   * uncache cannot reach them; a newer rebuild releases the oldest once its users return). */
  private val rebuilt = new java.util.ArrayDeque[String]()
  val MaxRebuilt = 2

  def put(key: String, rank: Int, state: Long): Unit = states.put((key, rank), new Entry(state))

  private def entry(key: String, rank: Int, source: Option[ReplaySource]): Entry = {
    val e = states.get((key, rank))
    if (e != null) e
    else if (rank == 0 && source.isDefined) rebuild(key, source.get)
    else throw new IllegalStateException(s"the GPU state of snapshot $key rank $rank is not resident on this executor")
  }

  /** Replays a single-GPU state's segment on this JVM's GPU (once per key, however many tasks ask);
   * the rebuilt state must hold the original's side sizes, or its ranges would not be the same rows. */
  private def rebuild(key: String, s: ReplaySource): Entry =
    rebuildLocks.computeIfAbsent(key, (_: String) => new Object).synchronized {
      val cur = states.get((key, 0))
      if (cur != null) cur
      else {
        val ctx = DeltaReplayContexts.forDevice(s.device)
        val staged = DeltaReplayNative.stageLog(ctx, s.logPath, s.version)
        val st = try DeltaReplayNative.replay(ctx, staged, s.minFileRetentionTs, s.validate)
                 finally DeltaReplayNative.stagedRelease(staged)
        val c = DeltaReplayNative.counts(st)
        import DeltaReplayNative.CountFields._
        if (c(NumFiles) != s.numFiles || c(NumRemoves) != s.numRemoves) {
          DeltaReplayNative.release(st)
          throw new IllegalStateException(s"the rebuilt GPU state of snapshot $key differs from the original " +
            s"(${c(NumFiles)}/${s.numFiles} files, ${c(NumRemoves)}/${s.numRemoves} tombstones)")
        }
        val e = new Entry(st)
        states.put((key, 0), e)
        rebuilt.synchronized {
          rebuilt.addLast(key)
          while (rebuilt.size > MaxRebuilt) release(rebuilt.pollFirst(), 0)
        }
        e
      }
    }

  /** Runs f on the state with a reference held: release waits for it (the state stays resident). With
   * a source, a state that is not resident here is rebuilt first (recompute lineage). */
  def use[T](key: String, rank: Int, source: Option[ReplaySource] = None)(f: Long => T): T = {
    val e = entry(key, rank, source)
    e.synchronized {
      if (e.released) throw new IllegalStateException(s"the GPU state of snapshot $key rank $rank was uncached")
      e.users += 1
    }
    try f(e.state)
    finally e.synchronized {
      e.users -= 1
      if (e.released && e.users == 0) DeltaReplayNative.release(e.state)
    }
  }

  /** Removes a rank's state and releases it (dr_state_release) now, or when its last user returns;
   * ranges already exported stay valid either way. */
  def release(key: String, rank: Int): Unit = {
    val e = states.remove((key, rank))
    if (e != null) e.synchronized {
      e.released = true
      if (e.users == 0) DeltaReplayNative.release(e.state)
    }
  }

  /** This executor's location for a partition that must run here (the rank's state lives here). */
  def here: String = {
    val bm = SparkEnv.get.blockManager.blockManagerId
    ExecutorCacheTaskLocation(bm.host, bm.executorId).toString
  }
}

/** Rows [lo, hi) of side `which` (Live / Tombstones) of rank `rank`'s state, preferably at `location`;
 * `source` (a single-GPU replay) lets any executor with a GPU rebuild the state. */
final case class StateRangePartition(index: Int, rank: Int, which: Int, lo: Long, hi: Long, location: String,
                                     source: Option[ReplaySource] = None)
  extends Partition

/** One rank's ranges: exportPlan of both sides on the rank's own executor. */
final case class RankPlan(rank: Int, location: String, live: Array[Long], tombstones: Array[Long],
                          source: Option[ReplaySource] = None)

object RankPlan {
  /** exportPlan of the state registered as (key, rank) in this JVM; `source` for a single-GPU replay
   * (its partitions can then be recomputed elsewhere). */
  def local(key: String, rank: Int, maxRows: Long, source: Option[ReplaySource] = None): RankPlan = {
    DeltaReplayStates.use(key, rank) { st =>
      RankPlan(rank, DeltaReplayStates.here,
        DeltaReplayNative.exportPlan(st, DeltaReplayNative.Live, maxRows, DeltaReplayNative.MaxBufferBytes),
        DeltaReplayNative.exportPlan(st, DeltaReplayNative.Tombstones, maxRows, DeltaReplayNative.MaxBufferBytes),
        source)
    }
  }
}

/** The SingleAction rows of planned row ranges, each computed where its rank's state is resident. */
class DeltaReplayStateRDD(sc: SparkContext, key: String, ranges: Array[StateRangePartition])
  extends RDD[InternalRow](sc, Nil) {

  override protected def getPartitions: Array[Partition] = ranges.map(p => p: Partition)

  override protected def getPreferredLocations(p: Partition): Seq[String] =
    Seq(p.asInstanceOf[StateRangePartition].location)

  override def compute(p: Partition, ctx: TaskContext): Iterator[InternalRow] = {
    val r = p.asInstanceOf[StateRangePartition]
    val handle = new Array[Long](1)
    // off the rank's executor: rebuilt from the log when the partition has a source, else a loud
    // failure; an uncache meanwhile waits for the export
    val cols = DeltaReplayStates.use(key, r.rank, r.source)(st =>
      DeltaReplayNative.exportRange(st, r.which, r.lo, r.hi, handle))
    ctx.addTaskCompletionListener[Unit](_ => DeltaReplayNative.rangeRelease(handle(0)))
    val toRow = DeltaReplayState.serializer()
    val actions: Iterator[SingleAction] =
      if (r.which == DeltaReplayNative.Live) SingleActionColumns.addFileIterator(cols).map(a => SingleAction(add = a))
      else SingleActionColumns.removeFileIterator(cols).map(rm => SingleAction(remove = rm))
    actions.map(a => toRow(a).copy())  // the serializer reuses its row
  }
}

object DeltaReplayState {
  private lazy val encoder = ExpressionEncoder[SingleAction]()

  def serializer(): ExpressionEncoder.Serializer[SingleAction] = encoder.createSerializer()

  /** Partitions of every rank's plan: live ranges, then tombstone ranges, rank by rank. */
  def partitions(plans: Seq[RankPlan]): Array[StateRangePartition] = {
    val out = Array.newBuilder[StateRangePartition]
    var i = 0
    for (pl <- plans.sortBy(_.rank); (which, b) <- Seq(DeltaReplayNative.Live -> pl.live,
                                                         DeltaReplayNative.Tombstones -> pl.tombstones)) {
      for (k <- 0 until b.length - 1) {
        out += StateRangePartition(i, pl.rank, which, b(k), b(k + 1), pl.location, pl.source)
        i += 1
      }
    }
    out.result()
  }

  /**
   * Snapshot.state (D/Snapshot.scala:120): the file actions of the resident ranks' states as
   * partitioned rows, plus the table-wide protocol / metaData / txn winners (a handful of actions,
   * nonFileJson decoded by Action.fromJson on the driver) in one more partition, wrapped as a
   * LogicalRDD exactly as CachedDS wraps the reference's cached RDD (D/util/StateCache.scala:56-62).
   */
  def dataset(spark: SparkSession, key: String, plans: Seq[RankPlan],
              nonFile: Seq[SingleAction]): Dataset[SingleAction] = {
    val sc = spark.sparkContext
    val files = new DeltaReplayStateRDD(sc, key, partitions(plans))
    val others = sc.parallelize(nonFile, 1).mapPartitions { it =>
      val toRow = serializer()
      it.map(a => toRow(a).copy())
    }
    val rdd = sc.union(files, others)
    rdd.setName(s"Delta GPU state $key")
    Dataset.ofRows(spark, LogicalRDD(encoder.schema.toAttributes, rdd)(spark)).as[SingleAction](encoder)
  }

  /**
   * The plans of a sharded replay: one task per rank on the executor holding it (the same tasks that
   * ran dr_replay_sharded registered their states under `key`), each returning exportPlan of both
   * sides. `locations(r)` is rank r's executor (recorded when the replay tasks ran).
   */
  def shardedPlans(sc: SparkContext, key: String, locations: IndexedSeq[String], maxRows: Long): Seq[RankPlan] = {
    val world = locations.size
    val ranks = new RDD[Int](sc, Nil) {
      override protected def getPartitions: Array[Partition] =
        Array.tabulate(world)(r => new Partition { override def index: Int = r })
      override protected def getPreferredLocations(p: Partition): Seq[String] = Seq(locations(p.index))
      override def compute(p: Partition, ctx: TaskContext): Iterator[Int] = Iterator(p.index)
    }
    ranks.map(r => RankPlan.local(key, r, maxRows)).collect().toSeq
  }
}
