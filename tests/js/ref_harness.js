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
const fs = require('fs');
const path = require('path');
const vm = require('vm');

const REF = process.env.APM_REF_DIR || '/root/reference';
const src = (f) => fs.readFileSync(path.join(REF, f), 'utf8');

function sliceBetween(text, startMarker, endMarker) {
  const a = text.indexOf(startMarker);
  if (a < 0) throw new Error('marker not found: ' + startMarker);
  const b = endMarker ? text.indexOf(endMarker, a + startMarker.length) : text.length;
  if (b < 0) throw new Error('marker not found: ' + endMarker);
  return text.slice(a, b);
}

function sliceFunction(text, startMarker) {
  const a = text.indexOf(startMarker);
  if (a < 0) throw new Error('marker not found: ' + startMarker);
  let i = text.indexOf('{', a);
  let depth = 0;
  for (; i < text.length; i++) {
    const c = text[i];
    if (c === '/' && text[i + 1] === '/') { i = text.indexOf('\n', i); if (i < 0) break; continue; }
    if (c === '/' && text[i + 1] === '*') { i = text.indexOf('*/', i + 2) + 1; continue; }
    if (c === '"' || c === "'" || c === '`') {
      for (i++; i < text.length && text[i] !== c; i++) if (text[i] === '\\') i++;
      continue;
    }
    if (c === '{') depth++;
    else if (c === '}') { depth--; if (depth === 0) return text.slice(a, i + 1); }
  }
  throw new Error('unbalanced: ' + startMarker);
}

const clock = { now: 0 };
const noop = () => {};
const logger = { info: noop, warn: noop, error: noop, debug: noop };

class NodeCacheStub {
  constructor(opts) { this.ttl = (opts && opts.stdTTL ? opts.stdTTL : 0) * 1000; this.data = new Map(); this.h = {}; }
  on(ev, fn) { this.h[ev] = fn; }
  _check(k) {
    const d = this.data.get(k);
    if (d.t !== 0 && d.t < clock.now) {
      this.data.delete(k);
      if (this.h.expired) this.h.expired(k, d.v);
      return false;
    }
    return true;
  }
  set(k, v) { this.data.set(k, { v, t: this.ttl ? clock.now + this.ttl : 0 }); return true; }
  get(k) { if (this.data.has(k) && this._check(k)) return this.data.get(k).v; return undefined; }
  has(k) { return this.data.has(k) && this._check(k); }
  sweep() { for (const k of Array.from(this.data.keys())) if (this.data.has(k)) this._check(k); }
  getStats() { return {}; }
}

const RealDate = Date;
class FakeDate extends RealDate {
  constructor(...args) { if (args.length === 0) super(clock.now); else super(...args); }
  static now() { return clock.now; }
}

function makeContext(extra) {
  const modules = {
    md5: (x) => String(x.length),
    nodemailer: { createTransport: () => ({ sendMail: async () => ({}) }) },
    sqlite3: { verbose: () => ({}) },
    fs, path,
  };
  const module = { exports: {} };
  const ctx = {
    require: (n) => { if (n in modules) return modules[n]; throw new Error('require ' + n); },
    module, exports: module.exports, console, logger, Math, JSON, parseFloat, parseInt, isNaN,
    setTimeout: noop, setInterval: noop, clearTimeout: noop, Promise, Map, Set,
    Date: FakeDate, Buffer, process: { on: noop, env: {} },
    NodeCache: NodeCacheStub,
  };
  Object.assign(ctx, extra || {});
  vm.createContext(ctx);
  // util_methods installs prototype helpers into this realm
  vm.runInContext(src('util_methods.js'), ctx, { filename: 'util_methods.js' });
  ctx.module.exports.call(ctx);
  // entries + heap
  const m1 = { exports: {} }; ctx.module = m1;
  vm.runInContext(src('entries.js'), ctx, { filename: 'entries.js' });
  Object.assign(ctx, m1.exports);
  ctx.entryFactory = new m1.exports.EntryFactory();
  const m2 = { exports: {} }; ctx.module = m2;
  vm.runInContext(src('binary_heap.js'), ctx, { filename: 'binary_heap.js' });
  ctx.BinaryHeap = m2.exports;
  return ctx;
}

function stripJSON(txt) { return txt.replace(new RegExp("[^:]\\/\\/(.*)", "g"), ''); }

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
  const fn = vm.runInContext('(function(){\n' + cls + '\nconst zscore = new ZScoreParser();\n' +
      'const entryFactory = new EntryFactory();\n' + consume + '\nreturn consumeMsg; })()', ctx,
      { filename: 'stream_calc_z_score.slice.js' });
  for (const line of req.lines) fn({ content: Buffer.from(line) });
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
  for (const line of req.lines) {
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
