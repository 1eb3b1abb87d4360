// Shared loader for the reference's own JavaScript (read from APM_REF_DIR, default
// /root/reference, never modified): slices classes/functions out of the stage scripts and runs
// them in a vm context with stubbed I/O, a clock-driven NodeCache and an injectable Date.now.
// Used by ref_harness.js (differential tests) and tools/reference_pipeline.js (CPU baseline).
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
// one Date class per context: util_methods.js installs non-configurable prototype methods
function makeFakeDate() {
  return class FakeDate extends RealDate {
    constructor(...args) { if (args.length === 0) super(clock.now); else super(...args); }
    static now() { return clock.now; }
  };
}
const FakeDate = makeFakeDate();

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
    Date: makeFakeDate(), Buffer, process: { on: noop, env: {} },
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


module.exports = { REF, src, sliceBetween, sliceFunction, clock, logger, NodeCacheStub, FakeDate, makeContext,
                   stripJSON, vm };
