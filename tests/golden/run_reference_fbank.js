// Runs the reference's own executable fbank -- computeFbank() of
// /root/reference/offline_pwa/static/js/pure-ort-asr-worker.js:470-519 (window :359-367,
// Hz-domain mel triangles :369-397, radix-2 FFT :399-458, reflection :460-468) -- under node,
// on raw float32 inputs, and writes its raw float32 outputs.  Test infrastructure only, run by
// tests/golden/make_golden_fbank_js.py in the build container (the reference is not on the
// GPU box).
//
// The worker file is evaluated as it is, in a vm context whose `self` / `importScripts` stand
// in for the Web Worker globals (importScripts throws, so the worker's onnxruntime-web set-up
// takes its own catch branch and nothing of ORT is touched).  The one change to its text:
// this container's node (v12) predates optional chaining, so `a?.b` / `a?.[k]` are rewritten
// to the equivalent `(a == null ? undefined : a.b)` before evaluation -- a syntax lowering
// that leaves every arithmetic operation of computeFbank as written.
//
// usage: node run_reference_fbank.js <worker.js> <in.f32> <lengths comma-separated> <out.f32>
"use strict";
const fs = require("fs");
const vm = require("vm");

const [workerPath, inPath, lensArg, outPath] = process.argv.slice(2);
let src = fs.readFileSync(workerPath, "utf8");
const chain = "([A-Za-z_$][\\w$]*(?:\\.[A-Za-z_$][\\w$]*)*)";
src = src.replace(new RegExp(chain + "\\?\\.\\[([^\\]]*)\\]", "g"),
                  "(($1) == null ? undefined : ($1)[$2])");
src = src.replace(new RegExp(chain + "\\?\\.([A-Za-z_$][\\w$]*)", "g"),
                  "(($1) == null ? undefined : ($1).$2)");
if (src.includes("?.")) throw new Error("optional chaining left after lowering");

const posted = [];
const ctx = {
  self: { postMessage: (m) => posted.push(m) },
  importScripts: () => { throw new Error("importScripts is not available (fbank run)"); },
  console,
};
vm.createContext(ctx);
vm.runInContext(src, ctx, { filename: workerPath });
if (typeof ctx.computeFbank !== "function") throw new Error("computeFbank not defined");

const raw = fs.readFileSync(inPath);
const all = new Float32Array(raw.buffer, raw.byteOffset, raw.byteLength / 4);
const lens = lensArg.split(",").map((x) => parseInt(x, 10));
const CtxF32 = vm.runInContext("Float32Array", ctx);  // the context realm's constructor
const outs = [];
let off = 0;
for (const n of lens) {
  const samples = CtxF32.from(all.subarray(off, off + n));
  off += n;
  const res = ctx.computeFbank(samples);
  if (res.data.length !== res.frames * 80) throw new Error("bad output size");
  outs.push(Buffer.from(new Float32Array(res.data).buffer));
}
fs.writeFileSync(outPath, Buffer.concat(outs));
process.stdout.write(JSON.stringify({ inputs: lens.length, samples: off, posted: posted.length }) + "\n");
