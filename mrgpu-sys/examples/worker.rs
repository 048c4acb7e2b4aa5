//! The reference worker's map and reduce tasks on the GPU (src/mr/worker.rs:142-193), with the
//! reference's file names: data/gut-{m}.txt in, mr-{r}.txt out.  Same calls as
//! tests/ffi/worker_harness.c, which the GPU tests run.
//!     cargo run --example worker -- <map_n> <reduce_n>
use mrgpu_sys::{Ctx, MRG_APP_WC};

fn main() -> Result<(), Box<dyn std::error::Error>> {
    let args: Vec<String> = std::env::args().collect();
    let map_n: u32 = args.get(1).map(|s| s.parse()).transpose()?.unwrap_or(6);
    let reduce_n: u32 = args.get(2).map(|s| s.parse()).transpose()?.unwrap_or(10);
    let ctx = Ctx::open(0)?;
    let mut parts = Vec::new();
    for m in 0..map_n {
        let name = format!("data/gut-{m}.txt");                     // worker.rs:67
        let contents = std::fs::read_to_string(&name)?;               // worker.rs:73-75
        parts.push(ctx.map(MRG_APP_WC, &contents, &name, m, reduce_n)?);
    }
    for r in 0..reduce_n {
        let bytes = ctx.reduce(MRG_APP_WC, r, &parts, reduce_n, &[])?;
        std::fs::write(format!("mr-{r}.txt"), bytes)?;                // worker.rs:167-179
    }
    Ok(())
}
