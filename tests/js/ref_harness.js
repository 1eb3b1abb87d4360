#!/usr/bin/env node
// Differential-test harness: executes the *reference's own* JavaScript (read from
// APM_REF_DIR, default /root/reference, never modified) inside a vm context with stubbed
// I/O, a clock-driven NodeCache and an injectable Date.now, and prints the records each stage
// emits. Input: one JSON request on stdin; output: one JSON response on stdout.
//
// Modes:
//   parse   {batches:[{now, chunks:[[path,[lines]]]}]}        -> [[queue, line], ...]
//   stats   {lines:[tx csv...]}                                 -> {st:[...], db:[...]}
//   zscore  {config, lines:[st csv...]}                         -> [fs csv...]
//   alerts  {config, lines:[fs csv...], clock:'entry'}          -> [al csv...]
//   util    {percentile:[[arr,p]...], average:[arr...], stddev:[arr...]}
'use strict';
const { src, sliceBetween, sliceFunction, clock, makeContext, stripJSON, vm } = require('./ref_lib.js');

function runParse(req) {
  const out = [];
  const q = (name) => ({ writeLineToQueue: (line) => out.push([name, line]) });
  const ctx = makeContext({ outQueue: q('transactions'), dbQueue: q('db_insert'),
                            PARSETXCONFIG: { verboseQueueWrite: false } });
  const body = sliceBetween(src('stream_parse_transactions.js'), 'const context = new Map();',
                            'logger.info(PARSETXCONFIG.maskSuffixes');
  const api = vm.runInContext('(function(){\n' + body +
      '\nreturn { readLine, acctCache, recordCache, needNumRecordCache };\n})()', ctx,
      { filename: 'stream_parse_transactions.slice.js' });
  const errors = [];
  for (const b of req.batches) {
    clock.now = b.now;
    api.recordCache.sweep(); api.needNumRecordCache.sweep(); api.acctCache.sweep();
    for (const [fp, lines] of b.chunks) {
      for (const line of lines) {
        try { api.readLine(fp, line); } catch (e) { errors.push(String(e)); }
      }
    }
  }
  return { records: out, errors };
}

function runStats(req) {
  const st = [], db = [];
  const ctx = makeContext({ CALCSTATSCONFIG: { verboseQueueWrite: false, logDebug: false } });
  const cls = sliceBetween(src('stream_calc_stats.js'), 'class StatParser', '//////////');
  const consume = sliceFunction(src('stream_calc_stats.js'), 'function consumeMsg(msg)');
  ctx.outQueue = { writeLineToQueue: (l) => st.push(l) };
  ctx.dbQueue = { writeLineToQueue: (l) => db.push(l) };
  const fn = vm.runInContext('(function(){\n' + cls + '\n' +
      'const INTERVAL_LENGTH_SEC=10, WINDOW_SZ=30, INTERVAL_BUFFER_SZ=6, NUM_KEEP_INTERVALS=36;\n' +
      'const data = new StatParser();\n' + consume + '\nreturn consumeMsg; })()', ctx,
      { filename: 'stream_calc_stats.slice.js' });
  for (const line of req.lines) fn({ content: Buffer.from(line) });
  return { st, db };
}

function runZScore(req) {
  const out = [];
  const cfg = JSON.parse(stripJSON(req.configText));
  const ctx = makeContext({ ZSCORECONFIG: cfg.streamCalcZScore });
  const cls = sliceBetween(src('stream_calc_z_score.js'), 'class ZScoreParser', '// async function writeStringToQueue');
  const consume = sliceFunction(src('stream_calc_z_score.js'), 'function consumeMsg(msg)');
  ctx.outQueue = { writeLineToQueue: (l) => out.push(l) };
  ctx.ZSCORECONFIG = { verboseQueueWrite: false, ...cfg.streamCalcZScore };
  const api = vm.runInContext('(function(){\n' + cls + '\nconst zscore = new ZScoreParser();\n' +
      'const entryFactory = new EntryFactory();\n' + consume + '\nreturn { consumeMsg, zscore }; })()', ctx,
      { filename: 'stream_calc_z_score.slice.js' });
  // reloads: [{at: line index, configText}] -- the watcher callback of stream_calc_z_score.js:
  // 362-382 (new ZSCORECONFIG, updateAllServiceSettings, removeStaleLagData) before line `at`
  const reloads = (req.reloads || []).slice().sort((a, b) => a.at - b.at);
  req.lines.forEach((line, i) => {
    while (reloads.length && reloads[0].at === i) {
      const c = JSON.parse(stripJSON(reloads.shift().configText));
      ctx.ZSCORECONFIG = { verboseQueueWrite: false, ...c.streamCalcZScore };
      api.zscore.updateAllServiceSettings();
      api.zscore.removeStaleLagData();
    }
    api.consumeMsg({ content: Buffer.from(line) });
  });
  return out;
}

function runAlerts(req) {
  const out = [];
  const cfg = JSON.parse(stripJSON(req.configText));
  const ctx = makeContext({ ALERTSCONFIG: cfg.streamProcessAlerts, APMCONFIG: cfg });
  const cls = sliceBetween(src('stream_process_alerts.js'), 'class AlertsManager', '// async function setUpDB');
  const mgr = vm.runInContext('(function(){\n' + cls + '\nreturn new AlertsManager(); })()', ctx,
      { filename: 'stream_process_alerts.slice.js' });
  const ef = new ctx.EntryFactory();
  // reloads: [{at, configText}] -- every gate is read from ALERTSCONFIG per entry, so a reload
  // is the new ALERTSCONFIG from line `at` on (stream_process_alerts.js:540-556)
  const reloads = (req.reloads || []).slice().sort((a, b) => a.at - b.at);
  for (let i = 0; i < req.lines.length; ++i) {
    const line = req.lines[i];
    while (reloads.length && reloads[0].at === i) {
      const c = JSON.parse(stripJSON(reloads.shift().configText));
      ctx.ALERTSCONFIG = c.streamProcessAlerts;
      ctx.APMCONFIG = c;
    }
    const en = ef.getEntryFromCSV(line);
    if (req.clock === 'entry') clock.now = en.timestamp;
    const al = mgr.processFSEntry(en);
    if (al) out.push(al.toCSVString());
  }
  return out;
}

function runUtil(req) {
  const ctx = makeContext({});
  const res = { percentile: [], average: [], stddev: [] };
  vm.runInContext('this.__mk = (a) => Array.from(a)', ctx);
  for (const [arr, p] of req.percentile || []) res.percentile.push(ctx.__mk(arr).calcPercentile(p));
  for (const arr of req.average || []) { const v = ctx.__mk(arr).average(); res.average.push(v === undefined ? null : v); }
  for (const arr of req.stddev || []) { const v = ctx.__mk(arr).standardDeviation(); res.stddev.push(v === undefined ? null : (Number.isNaN(v) ? 'NaN' : v)); }
  return res;
}

let input = '';
process.stdin.on('data', (d) => { input += d; });
process.stdin.on('end', () => {
  const req = JSON.parse(input);
  let res;
  if (req.mode === 'parse') res = runParse(req);
  else if (req.mode === 'stats') res = runStats(req);
  else if (req.mode === 'zscore') res = runZScore(req);
  else if (req.mode === 'alerts') res = runAlerts(req);
  else if (req.mode === 'util') res = runUtil(req);
  else throw new Error('unknown mode ' + req.mode);
  process.stdout.write(JSON.stringify(res));
});
