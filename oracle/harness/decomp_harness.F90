! =============================================================================
! decomp_harness -- TEST INFRASTRUCTURE ONLY (the "oracle", never the product)
!
! Runs the reference's own domain decomposition on a mesh given as raw arrays:
! the unmodified framework/mpas_block_decomp.F (cells of each block from a
! graph.info.part.N file, mpas_block_decomp_cells_for_proc) and
! framework/mpas_block_creator.F (owned cells, edges and vertices, their halo
! layers and exchange lists), called in the order mpas_bootstrapping.F:171-269
! calls them, on one MPI task holding every block or under mpirun.  It dumps, per block, the
! global index of every local element (indexTo*ID, owned first, then each halo
! layer), the per-layer end counts (n*Solve fields), and the exchange lists of
! the indexTo*ID fields, which pins mpas_dycore/decomp.py (tests/test_decomp_pinned.py).
!
! Usage: decomp_harness <input_dir> <output_dir>   (or under mpirun -np P: P tasks, the blocks dealt
!        out by mpas_block_decomp.F; tasks exchange through sendList / recvList instead of copyList)
!   <input_dir>/decomp.nml  namelist /decomp/ nCells, nEdges, nVertices, maxEdges, nblocks, nHalos
!   <input_dir>/{nEdgesOnCell,cellsOnCell,edgesOnCell,verticesOnCell,cellsOnEdge,cellsOnVertex}.bin
!     int32, MPAS 1-based (Fortran memory images without the garbage slot)
!   <input_dir>/graph.info.part.<nblocks>  (what mpas_block_decomp.F reads)
! =============================================================================
program decomp_harness
   use mpas_derived_types
   use mpas_pool_routines
   use mpas_kind_types
   use mpas_dmpar
   use mpas_log
   use mpas_block_decomp
   use mpas_block_creator
#ifdef DROPIN_PLAN
   use mpas_domain_routines, only : mpas_allocate_block
   use atm_time_integration, only : atm_dycore_plan_exchanges
#endif
   implicit none

   character(len=256) :: indir, outdir
   integer :: nCells, nEdges, nVertices, maxEdges, nblocks, nHalos, u, i
   integer :: cs, ce, es, ee, vs, ve   ! this task's read ranges (mpas_dmpar_get_index_range)
   integer, parameter :: vertexDegree = 3
   namelist /decomp/ nCells, nEdges, nVertices, maxEdges, nblocks, nHalos

   type (domain_type), pointer :: domain
   type (block_type), pointer :: readingBlock
   type (graph) :: partial_global_graph_info
   integer, dimension(:), pointer :: local_cell_list, block_id, block_start, block_count
   type (field1dInteger), pointer :: indexToCellIDField, nEdgesOnCellField, indexToEdgeIDField, indexToVertexIDField
   type (field2dInteger), pointer :: cellsOnCellField, edgesOnCellField, verticesOnCellField, cellsOnEdgeField, &
                                     cellsOnVertexField
   type (field1dInteger), pointer :: indexToCellID_Block, nEdgesOnCell_Block, indexToEdgeID_Block, &
                                     indexToVertexID_Block, nCellsSolveField, nEdgesSolveField, nVerticesSolveField
   type (field2dInteger), pointer :: cellsOnCell_Block, verticesOnCell_Block, edgesOnCell_Block, cellsOnEdge_Block, &
                                     cellsOnVertex_Block

   call get_command_argument(1, indir)
   call get_command_argument(2, outdir)
   nHalos = 2
   open(newunit=u, file=trim(indir)//'/decomp.nml', status='old')
   read(u, nml=decomp)
   close(u)

   allocate(domain)
   allocate(domain % dminfo)
   call mpas_dmpar_init(domain % dminfo)
   allocate(domain % core)
   domain % core % coreName = 'decomp'
   call mpas_log_init(domain % logInfo, domain)
   call mpas_log_open()

   ! ---- the "read" fields (mpas_io_setup_*_block_fields): each task reads its contiguous range of
   ! cells, edges and vertices, as mpas_bootstrapping.F:171-199 does ----
   call mpas_dmpar_get_index_range(domain % dminfo, 1, nCells, cs, ce)
   call mpas_dmpar_get_index_range(domain % dminfo, 1, nEdges, es, ee)
   call mpas_dmpar_get_index_range(domain % dminfo, 1, nVertices, vs, ve)
   allocate(readingBlock)
   readingBlock % domain => domain
   readingBlock % blockID = domain % dminfo % my_proc_id
   readingBlock % localBlockID = 0
   call read_field1(indexToCellIDField, '', cs, ce, nHalos)
   call read_field1(nEdgesOnCellField, 'nEdgesOnCell', cs, ce, -1, indexToCellIDField)
   call read_field2(cellsOnCellField, 'cellsOnCell', maxEdges, cs, ce, indexToCellIDField)
   call read_field2(edgesOnCellField, 'edgesOnCell', maxEdges, cs, ce, indexToCellIDField)
   call read_field2(verticesOnCellField, 'verticesOnCell', maxEdges, cs, ce, indexToCellIDField)
   call read_field1(indexToEdgeIDField, '', es, ee, nHalos + 1)
   call read_field2(cellsOnEdgeField, 'cellsOnEdge', 2, es, ee, indexToEdgeIDField)
   call read_field1(indexToVertexIDField, '', vs, ve, nHalos + 1)
   call read_field2(cellsOnVertexField, 'cellsOnVertex', vertexDegree, vs, ve, indexToVertexIDField)

   ! ---- mpas_bootstrapping.F:207-269 ----
   partial_global_graph_info % nVertices = ce - cs + 1
   partial_global_graph_info % nVerticesTotal = nCells
   partial_global_graph_info % maxDegree = maxEdges
   partial_global_graph_info % ghostStart = nVertices + 1
   allocate(partial_global_graph_info % vertexID(ce - cs + 1))
   allocate(partial_global_graph_info % nAdjacent(ce - cs + 1))
   allocate(partial_global_graph_info % adjacencyList(maxEdges, ce - cs + 1))
   partial_global_graph_info % vertexID(:) = indexToCellIDField % array(:)
   partial_global_graph_info % nAdjacent(:) = nEdgesOnCellField % array(:)
   partial_global_graph_info % adjacencyList(:,:) = cellsOnCellField % array(:,:)
   call mpas_block_decomp_cells_for_proc(domain % dminfo, partial_global_graph_info, local_cell_list, block_id, &
                                         block_start, block_count, nblocks, .false., &
                                         trim(indir)//'/graph.info.part.', '')
   call mpas_block_creator_setup_blocks_and_0halo_cells(nHalos, domain, indexToCellID_Block, local_cell_list, &
                                                        block_id, block_start, block_count)
   call mpas_block_creator_build_0halo_cell_fields(nHalos, indexToCellIDField, nEdgesOnCellField, cellsOnCellField, &
                                                   verticesOnCellField, edgesOnCellField, indexToCellID_Block, &
                                                   nEdgesOnCell_Block, cellsOnCell_Block, verticesOnCell_Block, &
                                                   edgesOnCell_Block)
   call mpas_block_creator_build_0_and_1halo_edge_fields(nHalos, indexToEdgeIDField, cellsOnEdgeField, &
                                                         indexToCellID_Block, nEdgesOnCell_Block, edgesOnCell_Block, &
                                                         indexToEdgeID_Block, cellsOnEdge_Block, nEdgesSolveField)
   call mpas_block_creator_build_0_and_1halo_edge_fields(nHalos, indexToVertexIDField, cellsOnVertexField, &
                                                         indexToCellID_Block, nEdgesOnCell_Block, verticesOnCell_Block, &
                                                         indexToVertexID_Block, cellsOnVertex_Block, nVerticesSolveField)
   call mpas_block_creator_build_cell_halos(nHalos, indexToCellID_Block, nEdgesOnCell_Block, cellsOnCell_Block, &
                                            verticesOnCell_Block, edgesOnCell_Block, nCellsSolveField)
   call mpas_block_creator_build_edge_halos(nHalos, indexToCellID_Block, nEdgesOnCell_Block, nCellsSolveField, &
                                            edgesOnCell_Block, indexToEdgeID_Block, cellsOnEdge_Block, nEdgesSolveField)
   call mpas_block_creator_build_edge_halos(nHalos, indexToCellID_Block, nEdgesOnCell_Block, nCellsSolveField, &
                                            verticesOnCell_Block, indexToVertexID_Block, cellsOnVertex_Block, &
                                            nVerticesSolveField)

   call dump_location('cell', indexToCellID_Block, nCellsSolveField)
   call dump_location('edge', indexToEdgeID_Block, nEdgesSolveField)
   call dump_location('vertex', indexToVertexID_Block, nVerticesSolveField)
#ifdef DROPIN_PLAN
   call plan_dropin()
#endif
   write(0, '(a)') 'decomp_harness: done'
   call mpas_dmpar_finalize(domain % dminfo)

contains

#ifdef DROPIN_PLAN
   ! Built as oracle/_ref/dropin_plan_harness (make -C oracle dropin_plan): the Fortran drop-in's
   ! domain-context path on this task's blocks, without a GPU (tests/test_dropin_multitask.py).  The
   ! blocks get what mpas_block_creator.F's finalize step gives them (:1000-1147): mpas_allocate_block,
   ! the pool dimensions, and parinfo's lists, which are the index fields' send / recv / copy lists;
   ! then the drop-in's atm_dycore_plan_exchanges writes <output_dir>/plan_task<rank>.txt.  The
   ! optional namelist /plan/ in decomp.nml holds the vertical size, scalars, dt and the namelist
   ! options that decide the exchange calls.
   subroutine plan_dropin()
      type (block_type), pointer :: b
      type (field1dInteger), pointer :: fc, fe, fv, sc, se, sv
      type (mpas_pool_type), pointer :: cfg, mesh, state
      character(len=320) :: path
      integer :: uu, ios
      integer :: nVertLevels, maxEdges2, num_scalars, moist_end, config_time_integration_order, &
                 config_number_of_sub_steps, config_dynamics_split_steps
      logical :: config_split_dynamics_transport, config_scalar_advection, config_monotonic, config_positive_definite
      real(kind=RKIND) :: dt
      namelist /plan/ nVertLevels, maxEdges2, num_scalars, moist_end, dt, config_time_integration_order, &
                      config_number_of_sub_steps, config_dynamics_split_steps, config_split_dynamics_transport, &
                      config_scalar_advection, config_monotonic, config_positive_definite
      nVertLevels = 26
      maxEdges2 = 2 * maxEdges
      num_scalars = 1
      moist_end = 1
      dt = 600.0_RKIND
      config_time_integration_order = 2
      config_number_of_sub_steps = 2
      config_dynamics_split_steps = 3
      config_split_dynamics_transport = .true.
      config_scalar_advection = .true.
      config_monotonic = .true.
      config_positive_definite = .false.
      open(newunit=uu, file=trim(indir)//'/decomp.nml', status='old')
      read(uu, nml=plan, iostat=ios)
      close(uu)
      call mpas_pool_create_pool(cfg)
      domain % configs => cfg
      call mpas_pool_add_config_int(cfg, 'config_time_integration_order', config_time_integration_order)
      call mpas_pool_add_config_int(cfg, 'config_number_of_sub_steps', config_number_of_sub_steps)
      call mpas_pool_add_config_int(cfg, 'config_dynamics_split_steps', config_dynamics_split_steps)
      call mpas_pool_add_config_int(cfg, 'config_number_rayleigh_damp_u_levels', 6)
      call mpas_pool_add_config_logical(cfg, 'config_split_dynamics_transport', config_split_dynamics_transport)
      call mpas_pool_add_config_logical(cfg, 'config_scalar_advection', config_scalar_advection)
      call mpas_pool_add_config_logical(cfg, 'config_positive_definite', config_positive_definite)
      call mpas_pool_add_config_logical(cfg, 'config_monotonic', config_monotonic)
      call mpas_pool_add_config_logical(cfg, 'config_mix_full', .true.)
      call mpas_pool_add_config_logical(cfg, 'config_rayleigh_damp_u', .true.)
      call mpas_pool_add_config_char(cfg, 'config_horiz_mixing', '2d_smagorinsky')
      call mpas_pool_add_config_real(cfg, 'config_h_mom_eddy_visc2', 0.0_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_h_mom_eddy_visc4', 0.0_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_v_mom_eddy_visc2', 0.0_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_h_theta_eddy_visc2', 0.0_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_h_theta_eddy_visc4', 0.0_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_v_theta_eddy_visc2', 0.0_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_len_disp', 120000.0_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_visc4_2dsmag', 0.05_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_del4u_div_factor', 10.0_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_coef_3rd_order', 0.25_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_smagorinsky_coef', 0.125_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_epssm', 0.1_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_smdiv', 0.1_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_apvm_upwinding', 0.5_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_mpas_cam_coef', 0.0_RKIND)
      call mpas_pool_add_config_real(cfg, 'config_rayleigh_damp_u_timescale_days', 5.0_RKIND)
      fc => indexToCellID_Block
      fe => indexToEdgeID_Block
      fv => indexToVertexID_Block
      sc => nCellsSolveField
      se => nEdgesSolveField
      sv => nVerticesSolveField
      do while (associated(fc))
         b => fc % block
         call mpas_allocate_block(nHalos, b, domain, b % blockID)
         b % parinfo % cellsToSend => fc % sendList
         b % parinfo % cellsToRecv => fc % recvList
         b % parinfo % cellsToCopy => fc % copyList
         b % parinfo % edgesToSend => fe % sendList
         b % parinfo % edgesToRecv => fe % recvList
         b % parinfo % edgesToCopy => fe % copyList
         b % parinfo % verticesToSend => fv % sendList
         b % parinfo % verticesToRecv => fv % recvList
         b % parinfo % verticesToCopy => fv % copyList
         call mpas_pool_create_pool(mesh)
         call mpas_pool_add_subpool(b % structs, 'mesh', mesh)
         call mpas_pool_create_pool(state)
         call mpas_pool_add_subpool(b % structs, 'state', state)
         call mpas_pool_add_dimension(mesh, 'nCells', sc % array(nHalos + 1))
         call mpas_pool_add_dimension(mesh, 'nEdges', se % array(nHalos + 2))
         call mpas_pool_add_dimension(mesh, 'nVertices', sv % array(nHalos + 2))
         call mpas_pool_add_dimension(mesh, 'nCellsSolve', sc % array(1))
         call mpas_pool_add_dimension(mesh, 'nEdgesSolve', se % array(1))
         call mpas_pool_add_dimension(mesh, 'nVerticesSolve', sv % array(1))
         call mpas_pool_add_dimension(mesh, 'nVertLevels', nVertLevels)
         call mpas_pool_add_dimension(mesh, 'maxEdges', maxEdges)
         call mpas_pool_add_dimension(mesh, 'maxEdges2', maxEdges2)
         call mpas_pool_add_dimension(state, 'num_scalars', num_scalars)
         call mpas_pool_add_dimension(state, 'moist_start', 1)
         call mpas_pool_add_dimension(state, 'moist_end', moist_end)
         call mpas_pool_add_dimension(state, 'index_qv', 1)
         fc => fc % next
         fe => fe % next
         fv => fv % next
         sc => sc % next
         se => se % next
         sv => sv % next
      end do
      write(path, '(a,a,i0,a)') trim(outdir), '/plan_task', domain % dminfo % my_proc_id, '.txt'
      call atm_dycore_plan_exchanges(domain, dt, trim(path))
   end subroutine plan_dropin
#endif

   ! elements s..e of a file of d1 int32 per element
   subroutine read_i(name, a, d1, s, e)
      character(len=*), intent(in) :: name
      integer, intent(in) :: d1, s, e
      integer, intent(out) :: a(d1 * (e - s + 1))
      integer :: uu
      open(newunit=uu, file=trim(indir)//'/'//name//'.bin', access='stream', form='unformatted', status='old')
      read(uu, pos=int(4, 8) * int(d1, 8) * int(s - 1, 8) + 1) a
      close(uu)
   end subroutine read_i

   ! a 1-d read field of elements s..e; name '' = the index field itself (s..e), which owns the
   ! exchange lists
   subroutine read_field1(f, name, s, e, nlayers, owner)
      type (field1dInteger), pointer :: f
      character(len=*), intent(in) :: name
      integer, intent(in) :: s, e, nlayers
      type (field1dInteger), pointer, optional :: owner
      integer :: j, n
      n = e - s + 1
      allocate(f)
      allocate(f % array(n))
      if (len(name) == 0) then
         f % array = [(j, j = s, e)]
         call mpas_dmpar_init_multihalo_exchange_list(f % sendList, nlayers)
         call mpas_dmpar_init_multihalo_exchange_list(f % recvList, nlayers)
         call mpas_dmpar_init_multihalo_exchange_list(f % copyList, nlayers)
      else
         call read_i(name, f % array, 1, s, e)
         f % sendList => owner % sendList
         f % recvList => owner % recvList
         f % copyList => owner % copyList
      end if
      f % dimSizes(1) = n
      f % block => readingBlock
      nullify(f % next)
   end subroutine read_field1

   subroutine read_field2(f, name, d1, s, e, owner)
      type (field2dInteger), pointer :: f
      character(len=*), intent(in) :: name
      integer, intent(in) :: d1, s, e
      type (field1dInteger), pointer :: owner
      integer :: n
      n = e - s + 1
      allocate(f)
      allocate(f % array(d1, n))
      call read_i(name, f % array, d1, s, e)
      f % dimSizes(1) = d1
      f % dimSizes(2) = n
      f % block => readingBlock
      f % sendList => owner % sendList
      f % recvList => owner % recvList
      f % copyList => owner % copyList
      nullify(f % next)
   end subroutine read_field2

   ! per block (global block id i): <out>/block<i>/<loc>_index.bin (global ids, local order), <loc>_solve.bin (end of
   ! the owned elements and of each halo layer), and every exchange list node of the index field:
   ! <loc>_<kind>_<layer>.bin = records (endPointID, nList, srcList(nList), destList(nList))
   subroutine dump_location(loc, idx, solve)
      character(len=*), intent(in) :: loc
      type (field1dInteger), pointer :: idx, solve
      type (field1dInteger), pointer :: fi, fs
      type (mpas_multihalo_exchange_list), pointer :: ml
      type (mpas_exchange_list), pointer :: node
      character(len=320) :: dir
      integer :: uu, kind, layer
      character(len=4), dimension(3), parameter :: kinds = ['send', 'recv', 'copy']
      fi => idx
      fs => solve
      do while (associated(fi))
         write(dir, '(a,a,i0)') trim(outdir), '/block', fi % block % blockID
         call execute_command_line('mkdir -p '//trim(dir))
         open(newunit=uu, file=trim(dir)//'/'//loc//'_index.bin', access='stream', form='unformatted', status='replace')
         write(uu) fi % array(1:fi % dimSizes(1))
         close(uu)
         open(newunit=uu, file=trim(dir)//'/'//loc//'_solve.bin', access='stream', form='unformatted', status='replace')
         write(uu) fs % array(1:fs % dimSizes(1))
         close(uu)
         do kind = 1, 3
            if (kind == 1) ml => fi % sendList
            if (kind == 2) ml => fi % recvList
            if (kind == 3) ml => fi % copyList
            do layer = 1, size(ml % halos)
               write(dir, '(a,a,i0,a,a,a,a,a,i0,a)') trim(outdir), '/block', fi % block % blockID, '/', loc, '_', &
                     kinds(kind), '_', layer, '.bin'
               open(newunit=uu, file=trim(dir), access='stream', form='unformatted', status='replace')
               node => ml % halos(layer) % exchList
               do while (associated(node))
                  write(uu) node % endPointID, node % nList, node % srcList(1:node % nList), node % destList(1:node % nList)
                  node => node % next
               end do
               close(uu)
            end do
         end do
         fi => fi % next
         fs => fs % next
      end do
   end subroutine dump_location

end program decomp_harness
