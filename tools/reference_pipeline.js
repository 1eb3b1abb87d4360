#!/usr/bin/env node
// CPU baseline: run the reference's own stage code (parse -> stats -> z-score -> alerts, sliced
// from /root/reference by tests/js/ref_lib.js, unmodified) in ONE node process with the
// RabbitMQ hops replaced by direct calls, and time it.  Removing the broker, the message acks
// and the five-process topology can only make the reference faster than its deployed form, so
// the throughput measured here is an upper bound on the reference -- a conservative baseline.
//
// Usage: node tools/reference_pipeline.js <corpus.txt> <apm_config.json> [warmupBatches]
// Corpus format: "#B <now_ms>" starts a batch, "#F <path>" switches the current file, any other
// line is a log line of the current file.
'use strict';
const fs = require('fs');
const path = require('path');
const lib = require(path.join(__dirname, '..', 'tests', 'js', 'ref_lib.js'));
const { src, sliceBetween, sliceFunction, clock, makeContext, stripJSON, vm } = lib;

const [corpusPath, cfgPath, warmArg] = process.argv.slice(2);
const cfg = JSON.parse(stripJSON(fs.readFileSync(cfgPath, 'utf8')));
const warmBatches = parseInt(warmArg || '2');

const counts = { lines: 0, tx: 0, audit_db: 0, released: 0, st: 0, fs: 0, al: 0, db_insert: 0, errors: 0 };

// ---- stage 4: alerts (consumeMsg forwards everything to db_insert, processes fs)
const actx = makeContext({ ALERTSCONFIG: { verboseQueueWrite: false, ...cfg.streamProcessAlerts }, APMCONFIG: cfg });
const acls = sliceBetween(src('stream_process_alerts.js'), 'class AlertsManager', '// async function setUpDB');
const aconsume = sliceFunction(src('stream_process_alerts.js'), 'function consumeMsg(msg)');
actx.dbQueue = { writeLineToQueue: () => { counts.db_insert++; } };
const alertsConsume = vm.runInContext('(function(){\n' + acls + '\nconst alertsManager = new AlertsManager();\n' +
    'alertsManager.addToAlertBuffer = function(){};\nconst entryFactory = new EntryFactory();\n' + aconsume +
    '\nreturn consumeMsg; })()', actx, { filename: 'stream_process_alerts.slice.js' });

// ---- stage 3: z-score
const zctx = makeContext({ ZSCORECONFIG: { verboseQueueWrite: false, ...cfg.streamCalcZScore } });
const zcls = sliceBetween(src('stream_calc_z_score.js'), 'class ZScoreParser', '// async function writeStringToQueue');
const zconsume = sliceFunction(src('stream_calc_z_score.js'), 'function consumeMsg(msg)');
zctx.outQueue = { writeLineToQueue: (l) => { counts.fs++; alertsConsume({ content: Buffer.from(l) }); } };
const zscoreConsume = vm.runInContext('(function(){\n' + zcls + '\nconst zscore = new ZScoreParser();\n' +
    'const entryFactory = new EntryFactory();\n' + zconsume + '\nreturn consumeMsg; })()', zctx,
    { filename: 'stream_calc_z_score.slice.js' });

// ---- stage 2: stats
const sctx = makeContext({ CALCSTATSCONFIG: { verboseQueueWrite: false, logDebug: false } });
const scls = sliceBetween(src('stream_calc_stats.js'), 'class StatParser', '//////////');
const sconsume = sliceFunction(src('stream_calc_stats.js'), 'function consumeMsg(msg)');
sctx.outQueue = { writeLineToQueue: (l) => { counts.st++; zscoreConsume({ content: Buffer.from(l) }); } };
sctx.dbQueue = { writeLineToQueue: () => { counts.released++; } };
const statsConsume = vm.runInContext('(function(){\n' + scls + '\n' +
    'const INTERVAL_LENGTH_SEC=10, WINDOW_SZ=30, INTERVAL_BUFFER_SZ=6, NUM_KEEP_INTERVALS=36;\n' +
    'const data = new StatParser();\n' + sconsume + '\nreturn consumeMsg; })()', sctx,
    { filename: 'stream_calc_stats.slice.js' });

// ---- stage 1: parse
const pctx = makeContext({
  outQueue: { writeLineToQueue: (l) => { counts.tx++; statsConsume({ content: Buffer.from(l) }); } },
  dbQueue: { writeLineToQueue: () => { counts.audit_db++; } },
  PARSETXCONFIG: { verboseQueueWrite: false },
});
const body = sliceBetween(src('stream_parse_transactions.js'), 'const context = new Map();',
                          'logger.info(PARSETXCONFIG.maskSuffixes');
const api = vm.runInContext('(function(){\n' + body +
    '\nreturn { readLine, acctCache, recordCache, needNumRecordCache };\n})()', pctx,
    { filename: 'stream_parse_transactions.slice.js' });

// ---- corpus
const text = fs.readFileSync(corpusPath, 'utf8');
const lines = text.split('\n');
const batches = [];
let cur = null, file = null;
for (const ln of lines) {
  if (ln.startsWith('#B ')) { cur = { now: Number(ln.slice(3)), items: [] }; batches.push(cur); continue; }
  if (ln.startsWith('#F ')) { file = ln.slice(3); continue; }
  if (ln.length && cur) cur.items.push(file, ln);
}

function runBatch(b) {
  clock.now = b.now;
  api.recordCache.sweep(); api.needNumRecordCache.sweep(); api.acctCache.sweep();
  const it = b.items;
  for (let i = 0; i < it.length; i += 2) {
    counts.lines++;
    try { api.readLine(it[i], it[i + 1]); } catch (e) { counts.errors++; }
  }
}

for (let i = 0; i < Math.min(warmBatches, batches.length); i++) runBatch(batches[i]);
const c0 = Object.assign({}, counts);
const t0 = process.hrtime.bigint();
for (let i = warmBatches; i < batches.length; i++) runBatch(batches[i]);
const dt = Number(process.hrtime.bigint() - t0) / 1e9;
const d = {};
for (const k of Object.keys(counts)) d[k] = counts[k] - c0[k];
process.stdout.write(JSON.stringify({ seconds: dt, batches: batches.length - warmBatches, ...d,
  lines_per_s: d.lines / dt, tx_per_s: d.tx / dt, node: process.version }) + '\n');
